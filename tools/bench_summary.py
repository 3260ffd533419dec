"""One line per bench JSON log: ms per step, value, score_batch us per launch, solve ms
per launch, batch wait, solved/accepted.  usage: python tools/bench_summary.py LOG..."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            r, s = d.get("roofline", {}) or {}, d.get("speculation", {}) or {}
            print(f"{f:40s} ms {d['ms_per_step']:.3f} value {d['value']:.4g} score_us {r.get('avg_launch_us', 0):.1f} "
                  f"solve_ms {r.get('solve_ms_per_launch', 0):.3f} wait {d.get('ms_per_pair', {}).get('batch_wait', 0):.2f} "
                  f"solved/acc {s.get('solved_over_accepted', 0):.3f}")
