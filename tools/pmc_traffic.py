"""Fold the FETCH_SIZE / WRITE_SIZE passes of tools/measure.sh into profiles/pmc_traffic.json,
which bench.py reads for roofline.traffic (rocprofv3 cannot run inside the bench process).

usage: python tools/pmc_traffic.py gpurun_out/measure profiles/<round dir>
Copies the counter CSVs to <round dir>/pmc/ and writes one entry per topology, keyed
'k_persist|<bench workload string>'.
"""
import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CORR = ("FETCH_SIZE x2 (MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE tallies the 128-B "
        "memory requests of coalesced reads at 64 B); the dominant stream is the [S][B][4H] P1 "
        "stream (16-B loads) for k_persist_wide / k_persist_rr / k_persist_gen and, for k_persist "
        "(P1 formed in-kernel), the Gumbel noise (4-B lane loads, 256 B per wave) plus the per-frame "
        "tables; WRITE_SIZE as reported")
# workload -> (bench.py arguments as in tools/measure.sh ARGS, bench workload string, kernel key)
def workload(model, wname, frames=1000, utts=1, target=11000, overlap=550):
    return (f'{utts}x{frames}-frame mel per GPU, {model} {wname}, '
            f'batched folds target={target} overlap={overlap}')


WORKLOADS = {
    'c2': ('', workload('fatchord-wavernn', 'RAW 9-bit mu-law'), 'k_persist'),
    'c4': (' --utts-per-gpu 8', workload('fatchord-wavernn', 'RAW 9-bit mu-law', utts=8), 'k_persist_wide'),
    'c3': (' --mode MOL', workload('fatchord-wavernn', 'MOL'), 'k_persist'),
    'rr': (' --model runtimeracer-wavernn --bits 9', workload('runtimeracer-wavernn', 'RAW 9-bit mu-law'),
           'k_persist'),
    'gen': (' --model geneing-wavernn --mode BITS --bits 10', workload('geneing-wavernn', 'BITS 10-bit'),
            'k_persist'),
}


def counter(path, kernel):
    def base(name):  # 'void wrnn::k_persist<3, false>(wrnn::PersistArgs)' -> 'k_persist'
        return name.split('(')[0].split('<')[0].split('::')[-1]
    rows = [r for r in csv.DictReader(open(path)) if base(r['Kernel_Name']) == kernel]
    return rows[0]['Kernel_Name'], sum(float(r['Counter_Value']) for r in rows), len(rows)


def main():
    src, out = sys.argv[1:3]
    os.makedirs(os.path.join(out, 'pmc'), exist_ok=True)
    jpath = os.path.join(REPO, 'profiles', 'pmc_traffic.json')
    table = json.load(open(jpath)) if os.path.exists(jpath) else {}
    for key, (extra, wl, kernel) in WORKLOADS.items():
        f = os.path.join(src, f'pmc_fetch_{key}', 'run_counter_collection.csv')
        w = os.path.join(src, f'pmc_write_{key}', 'run_counter_collection.csv')
        if not (os.path.exists(f) and os.path.exists(w)):
            continue
        kname, fetch, n = counter(f, kernel)
        _, write, _ = counter(w, kernel)
        dst_f = os.path.join(out, 'pmc', f'fetch_size_{key}.csv')
        dst_w = os.path.join(out, 'pmc', f'write_size_{key}.csv')
        shutil.copy(f, dst_f)
        shutil.copy(w, dst_w)
        traffic = (2 * fetch + write) * 1024.0 / n  # KiB counters, per launch
        table[f'{kernel}|{wl}'] = {
            'kernel': kname, 'launches': n, 'fetch_size_kib': fetch / n, 'write_size_kib': write / n,
            'traffic_bytes': traffic, 'correction': CORR,
            'source': f'{os.path.relpath(dst_f, REPO)}, {os.path.relpath(dst_w, REPO)}: rocprofv3 '
                      f'--pmc FETCH_SIZE | WRITE_SIZE (separate passes) --kernel-include-regex '
                      f'{kernel} -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 '
                      f'--no-timing{extra}'}
        print(key, kname, f'{traffic / 1e9:.3f} GB per launch')
    json.dump(table, open(jpath, 'w'), indent=1)


if __name__ == '__main__':
    main()
