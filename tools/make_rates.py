"""Emit the launch planner's rate table from a measurement pass's bench lines.

Usage: python tools/make_rates.py OUT.txt DIR [DIR ...]

Reads the bench JSON lines of the probes tools/measure_r06.sh writes (each at a forced rows per
group, WRNN_PERSIST_NR_MAX=k and no rotation / slicing, so `us_per_step` is that variant's step
time) and writes `key v1 .. v4` lines for the keys it found; the runtime
(runtime.hip load_rates) overrides those keys of its built-in defaults and keeps the rest:
  <dir>/nr<k>.log      -> fat9      (fatchord 9-bit, C2 shape)
  <dir>/u10_nr<k>.log  -> fat10     (fatchord 10-bit, its 3000 / 1500 default)
  <dir>/sp_nr<k>.log   -> fat9_sp   (sparse instances, 90 %-pruned weights)
  <dir>/rr_nr<k>.log   -> rr        <dir>/gen_nr<k>.log -> gen
  <dir>/c4.log (16 rows / group, 512 classes), <dir>/b10.log (16 rows, 1024 classes),
  <dir>/u10_wide.log (6 rows, 1024 classes) -> wide = base, per row, 1024-class extra
Later directories override earlier ones. The rotation tables keep the runtime's defaults unless
a key is already in the file given as OUT (kept lines are carried over).
"""
import json
import os
import sys

FAMILIES = {'nr': 'fat9', 'u10_nr': 'fat10', 'sp_nr': 'fat9_sp', 'rr_nr': 'rr', 'gen_nr': 'gen'}


def line_of(path):
    try:
        for ln in open(path):
            if ln.startswith('{'):
                return json.loads(ln)
    except OSError:
        return None
    return None


def us_step(d):
    r = (d or {}).get('roofline') or {}
    return r.get('us_per_step')


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    keys, src = {}, {}
    for d in dirs:
        for pre, key in FAMILIES.items():
            vals = [us_step(line_of(os.path.join(d, f'{pre}{k}.log'))) for k in (1, 2, 3, 4)]
            if all(v is not None for v in vals):
                keys[key] = [round(v, 3) for v in vals]
                src[key] = d
        c4, b10, u10w = (us_step(line_of(os.path.join(d, f))) for f in ('c4.log', 'b10.log', 'u10_wide.log'))
        if c4 and b10:
            extra = b10 - c4
            per_row = ((b10 - extra) - (u10w - extra)) / 10.0 if u10w else 0.025
            per_row = max(per_row, 0.001)
            keys['wide'] = [round(c4 - 16 * per_row, 3), round(per_row, 4), round(extra, 3)]
            src['wide'] = d
    kept = []
    if os.path.exists(out):
        for ln in open(out):
            k = ln.split('#')[0].split()
            if k and k[0] not in keys:
                kept.append(ln.rstrip('\n'))
    with open(out, 'w') as f:
        f.write('# MI355X launch-planner rates (us per step), written by tools/make_rates.py from\n')
        for k in sorted(keys):
            f.write(f'#   {k}: {src[k]}\n')
        for k in sorted(keys):
            f.write(k + ' ' + ' '.join(str(v) for v in keys[k]) + '\n')
        for ln in kept:
            if not ln.startswith('#'):
                f.write(ln + '\n')
    print(open(out).read())


if __name__ == '__main__':
    main()
