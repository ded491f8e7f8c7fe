"""Turn a rocprofv3 --kernel-trace --stats CSV into the markdown table kept under profiles/.

usage: python tools/prof_summary.py <run_kernel_stats.csv> <out_dir> "<title>" "<command>"
"""
import csv
import os
import shutil
import sys


def main():
    src, out, title, cmd = sys.argv[1:5]
    os.makedirs(out, exist_ok=True)
    rows = list(csv.DictReader(open(src)))
    lines = [f'# {title}', '', f'Command: `{cmd}`', '',
             '| kernel | calls | avg us | min us | max us | total ms |', '|---|---|---|---|---|---|']
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
        lines.append(f"| {r['Name'][:70]} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.3f} | "
                     f"{float(r['MinNs']) / 1e3:.3f} | {float(r['MaxNs']) / 1e3:.3f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.3f} |")
    open(os.path.join(out, 'summary.md'), 'w').write('\n'.join(lines) + '\n')
    shutil.copy(src, os.path.join(out, 'kernel_stats.csv'))
    dom = src.replace('kernel_stats', 'domain_stats')
    if os.path.exists(dom):
        shutil.copy(dom, os.path.join(out, 'domain_stats.csv'))


if __name__ == '__main__':
    main()
