"""Print a compact view of bench.py JSON lines (timeline thinned)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        lines = [l for l in open(f).read().splitlines() if l.startswith("{")]
        d = json.loads(lines[-1])
    except Exception as ex:  # noqa: BLE001
        print(f, "unreadable:", ex)
        print(open(f).read()[-3000:])
        continue
    tl = d.pop("timeline", [])
    print(f)
    print(json.dumps(d)[:2500])
    for e in tl[:: max(1, len(tl) // 12)]:
        print({k: (round(v, 4) if isinstance(v, float) else v) for k, v in e.items()})
