"""Write <round dir>/summary.md from a tools/measure_r05.sh pass (bench lines, PMC fold, kernel stats).

usage: python tools/final_summary.py <pass dir> <round dir> <tag> [<round name>]
"""
import csv
import json
import os
import sys

LINES = ('bench', 'c4', 'rr', 'b10', 'c3', 'gen', 'gen_norot', 'gen_mol', 'rr_mol', 'rr9',
         'u10', 'spc2_auto', 'spc2', 'spc4')


def bench_line(path):
    if not os.path.exists(path):
        return None
    for line in open(path):
        if line.startswith('{'):
            return json.loads(line)
    return None


def main():
    src, out, tag = sys.argv[1:4]
    tests = open(os.path.join(src, 'tests.log')).read() if os.path.exists(os.path.join(src, 'tests.log')) else ''
    passed = [l for l in tests.splitlines() if ' passed' in l and '====' in l]
    rnd = sys.argv[4] if len(sys.argv) > 4 else 'Round-5'
    L = [f'# {rnd} final measurement pass (MI355X)', '',
         f'`tools/measure_r0{rnd[-1]}.sh` (TAG={tag}) on the final library build; GPU tests `tests.log` '
         f'({passed[-1].strip("= ") if passed else "see log"}), smoke `smoke.log`; counters `pmc/` (folded into '
         '`profiles/pmc_traffic.json`); kernel stats `prof_*/run_kernel_stats.csv`.', '',
         '| line | workload | value (samples/s) | ms / call | dominant kernel | us / launch step | '
         'call us / step of S | launches | HBM GB / launch (PMC) | MFMA busy | latency frac (idle / loaded floor) |',
         '|---|---|---|---|---|---|---|---|---|---|---|']
    c2 = None
    for name in LINES:
        d = bench_line(os.path.join(src, f'{name}.log'))
        if d is None:
            continue
        r = d['roofline']
        if name == 'bench':
            c2 = d
        wl = d['config']['workload'] + (' (rotation off)' if name == 'gen_norot' else '')
        tr = f"{r['traffic'] / 1e9:.3f}" if r.get('traffic') else 'n/a'
        if name.endswith('_norot'):  # (the counters are filed by workload: the rotated plan's launch)
            tr = 'n/a'
        mb = f"{r['mfma_busy_frac']:.2f}" if 'mfma_busy_frac' in r else 'n/a'
        L.append(f"| {name} | {wl} | {d['value']:,.0f} | {d['ms_per_step']:.2f} | {r['kernel']} | "
                 f"{r['us_per_step']:.3f} | {r['call_us_per_step']:.3f} | {r['launches_per_generate']} | {tr} | {mb} | "
                 f"{r['latency_frac']:.3f} / {r['latency_frac_loaded']:.3f} |")
    L.append('')
    if c2:
        r = c2['roofline']
        L.append(f"lib_build {c2['config']['lib_build']}, traffic_from_benched_build {r.get('traffic_from_benched_build')}.")
        cb = c2['cpu_baseline']
        legs = cb.get('legs', [])
        one = [g for g in legs if g['cores'] == 1]
        L.append(f"C2 CPU baseline (oracle, {cb.get('cpu_model')}): {cb['value']:,.0f} samples/s on {cb['cores']} threads"
                 + (f", {one[0]['value']:,.0f} on 1." if one else '.'))
        p = c2['parity']
        lg = p['logits']
        L.append(f"C2 parity in the timed call: labels_equal {p['labels_equal']}, wave_bit_exact {p['wave_bit_exact']}, "
                 f"max |dlogit| {lg['max_abs_logit_err']:.3g}, min top-2 gap / err {lg['gap_over_err']:.1f}.")
    for w in ('c2', 'c4', 'rr', 'b10'):
        f = os.path.join(src, f'prof_{w}', 'run_kernel_stats.csv')
        if not os.path.exists(f):
            continue
        rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
        r0 = rows[0]
        L.append(f"rocprof {w}: {r0['Name'][:60]} x{r0['Calls']} avg {float(r0['AverageNs']) / 1e6:.3f} ms")
    os.makedirs(out, exist_ok=True)
    open(os.path.join(out, 'summary.md'), 'w').write('\n'.join(L) + '\n')
    print('\n'.join(L))


if __name__ == '__main__':
    main()
