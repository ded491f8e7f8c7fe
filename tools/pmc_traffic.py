"""Fold rocprofv3 counter passes into profiles/pmc_traffic.json, which bench.py reads for
roofline.traffic and the counter-backed fractions (rocprofv3 cannot run inside the bench process).

usage: python tools/pmc_traffic.py <pass dir> <round dir> [<table json>]
  <pass dir>: tools/pmc_r03.sh output (gpurun_out/pmc3): <w>_fetch/, <w>_write/, <w>_sq/ per
              workload w (c2, c4, ...), each with run_counter_collection.csv, and lib_build
              (the SHA-256 prefix of the library the passes ran, bench.lib_build_id)
  <table json>: where to write the table (default profiles/pmc_traffic.json; the measurement
              script folds on the box into gpurun_out/ and points the bench at it)
Copies the CSVs to <round dir>/pmc/ and writes one entry per workload, keyed
'<kernel>|<bench workload string>', with per-launch values of the dominant kernel:
  traffic_bytes   HBM bytes: FETCH_SIZE x 2 + WRITE_SIZE (KiB counters; MI355X_MICROARCH.md HBM
                  section: gfx950 FETCH_SIZE tallies the 128-B requests of coalesced reads at 64 B)
  mfma_busy_frac  SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles), kernel cycles =
                  GRBM_GUI_ACTIVE / 8 (GRBM is summed over the 8 XCDs); the busy counter counts
                  MFMA pipe cycles (32 per v_mfma_f32_16x16x4_f32, MI355X_MICROARCH.md)
  lds_conflict_frac  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles / all LDS cycles)
  wait_frac, issue_stall_frac, active_frac  SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY
                  over SQ_WAVE_CYCLES (disjoint, MI355X_MICROARCH.md PMC table)
"""
import collections
import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CORR = ("FETCH_SIZE x2 (MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE tallies the 128-B "
        "memory requests of coalesced reads at 64 B); WRITE_SIZE as reported")
N_SIMD = 1024


def workload(model, wname, frames=1000, utts=1, target=11000, overlap=550, prune=0.0):
    return (f'{utts}x{frames}-frame mel per GPU, {model} {wname}, '
            f'batched folds target={target} overlap={overlap}' +
            (f', weights pruned {prune:.2f} in 1x4 blocks' if prune else ''))


# workload -> (bench.py arguments as in tools/pmc_r03.sh ARGS, bench workload string, kernel)
WORKLOADS = {
    'c2': ('', workload('fatchord-wavernn', 'RAW 9-bit mu-law'), 'k_persist'),
    'c4': (' --utts-per-gpu 8', workload('fatchord-wavernn', 'RAW 9-bit mu-law', utts=8), 'k_persist_wide'),
    'c3': (' --mode MOL', workload('fatchord-wavernn', 'MOL'), 'k_persist'),
    'b10': (' --bits 10 --target 3000 --overlap 1500 --utts-per-gpu 8',
            workload('fatchord-wavernn', 'RAW 10-bit mu-law', utts=8, target=3000, overlap=1500),
            'k_persist_wide'),
    'rr': (' --model runtimeracer-wavernn --bits 10 --target 6000 --overlap 1000 --utts-per-gpu 8',
           workload('runtimeracer-wavernn', 'RAW 10-bit mu-law', utts=8, target=6000, overlap=1000),
           'k_persist_wide_rr'),
    'gen': (' --model geneing-wavernn --mode BITS --bits 10',
            workload('geneing-wavernn', 'BITS 10-bit'), 'k_persist_gen'),
    # round 6: the fork's fatchord 10-bit single utterance (one wide launch of 6 rows per group)
    # and C2 on 90 %-pruned weights with the sparse instances forced
    'u10': (' --bits 10 --target 3000 --overlap 1500',
            workload('fatchord-wavernn', 'RAW 10-bit mu-law', target=3000, overlap=1500), 'k_persist_wide'),
    'spc2': (' --prune 0.9 --sparse 1', workload('fatchord-wavernn', 'RAW 9-bit mu-law', prune=0.9),
             'k_persist'),
}
# the table key's kernel name where it differs from the counted kernel's (bench.py roofline.kernel)
TABLE_KERNEL = {'spc2': 'k_persist (sparse)'}


def base(name):  # 'void wrnn::k_persist<3, false>(wrnn::PersistArgs)' -> 'k_persist'
    return name.split('(')[0].split('<')[0].split('::')[-1]


def per_launch(path, kernel):
    """{counter: value per launch} of `kernel` (summed over the dimension rows of a dispatch,
    averaged over dispatches), its full name and the dispatch count."""
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    name = None
    for r in csv.DictReader(open(path)):
        if base(r['Kernel_Name']) != kernel:
            continue
        name = r['Kernel_Name']
        disp[r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
    n = len(disp)
    tot = collections.defaultdict(float)
    for c in disp.values():
        for k, v in c.items():
            tot[k] += v
    return {k: v / n for k, v in tot.items()}, name, n


def main():
    src, out = sys.argv[1:3]
    os.makedirs(os.path.join(out, 'pmc'), exist_ok=True)
    jpath = os.path.join(REPO, 'profiles', 'pmc_traffic.json')
    table = json.load(open(jpath)) if os.path.exists(jpath) else {}
    if len(sys.argv) > 3:
        jpath = sys.argv[3]
    lib_build = None
    if os.path.exists(os.path.join(src, 'lib_build')):
        lib_build = open(os.path.join(src, 'lib_build')).read().strip() or None
    for key, (extra, wl, kernel) in WORKLOADS.items():
        paths = {p: os.path.join(src, f'{key}_{p}', 'run_counter_collection.csv')
                 for p in ('fetch', 'write', 'sq')}
        if not (os.path.exists(paths['fetch']) and os.path.exists(paths['write'])):
            continue
        for p, f in paths.items():
            if os.path.exists(f):
                shutil.copy(f, os.path.join(out, 'pmc', f'{key}_{p}.csv'))
        fetch, kname, n = per_launch(paths['fetch'], kernel)
        write, _, _ = per_launch(paths['write'], kernel)
        traffic = (2 * fetch['FETCH_SIZE'] + write['WRITE_SIZE']) * 1024.0
        rel = os.path.relpath(os.path.join(out, 'pmc'), REPO)
        e = {'kernel': kname, 'launches': n, 'lib_build': lib_build, 'fetch_size_kib': fetch['FETCH_SIZE'],
             'write_size_kib': write['WRITE_SIZE'], 'traffic_bytes': traffic, 'correction': CORR,
             'source': f'{rel}/{key}_fetch.csv, {rel}/{key}_write.csv: rocprofv3 --pmc FETCH_SIZE | '
                       f'WRITE_SIZE (separate passes) --kernel-include-regex {kernel} -- python3 '
                       f'bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-timing{extra}'}
        if os.path.exists(paths['sq']):
            sq, _, _ = per_launch(paths['sq'], kernel)
            cyc = sq['GRBM_GUI_ACTIVE'] / 8.0
            wc = sq['SQ_WAVE_CYCLES']
            e['counters'] = {k: sq[k] for k in sorted(sq)}
            e['kernel_cycles'] = cyc
            e['mfma_busy_frac'] = sq['SQ_VALU_MFMA_BUSY_CYCLES'] / (N_SIMD * cyc)
            e['lds_conflict_frac'] = (sq['SQ_LDS_BANK_CONFLICT'] / sq['SQ_LDS_IDX_ACTIVE']
                                      if sq['SQ_LDS_IDX_ACTIVE'] else 0.0)
            e['wait_frac'] = sq['SQ_WAIT_ANY'] / wc
            e['issue_stall_frac'] = sq['SQ_WAIT_INST_ANY'] / wc
            e['active_frac'] = sq['SQ_ACTIVE_INST_ANY'] / wc
            e['sq_source'] = (f'{rel}/{key}_sq.csv: rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES '
                              f'SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES '
                              f'SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE (one pass)')
        table[f'{TABLE_KERNEL.get(key, kernel)}|{wl}'] = e
        print(key, kname, f'{traffic / 1e9:.3f} GB per launch',
              {k: round(e[k], 3) for k in ('mfma_busy_frac', 'lds_conflict_frac', 'wait_frac') if k in e})
    json.dump(table, open(jpath, 'w'), indent=1)


if __name__ == '__main__':
    main()
