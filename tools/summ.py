"""One line per bench log: value, ms/step, dominant kernel, us per launch step, launches."""
import json
import sys

for p in sys.argv[1:]:
    for line in open(p):
        if not line.startswith('{'):
            continue
        d = json.loads(line)
        r = d.get('roofline') or {}
        sp = d['config'].get('sparse', {})
        print(f"{p.split('/')[-1]:22s} {d['value'] / 1e6:7.3f} M  {d['ms_per_step']:8.2f} ms  "
              f"{r.get('kernel', '-'):20s} us/step {r.get('us_per_step', 0):7.3f} call {r.get('call_us_per_step', 0):7.3f} "
              f"launches {r.get('launches_per_generate', '-')} sparse {sp.get('ran')} "
              f"rot {(r.get('rotation') or {}).get('launches', 0)} lat {r.get('latency_frac', 0):.3f}")
