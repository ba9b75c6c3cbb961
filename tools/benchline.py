"""One-line summary of bench.py JSON lines on stdin: python tools/benchline.py LABEL"""
import json
import sys

label = sys.argv[1] if len(sys.argv) > 1 else ""
for line in sys.stdin:
    r = json.loads(line)
    lds = (r.get("roofline_lds") or {}).get("frac")
    iss = r["roofline_issue"]["frac"]
    print(f"{label[:70]:70s} {r['value']/1e9:9.1f} G/s launch {r['roofline_hbm']['launch_us']:8.1f}us "
          f"issue {'-' if iss is None else format(iss, '.3f')} hbm {r['roofline_hbm']['frac']:.3f} "
          f"lds {'-' if lds is None else format(lds, '.3f')} {r['config'].get('executor','')[:60]}")
