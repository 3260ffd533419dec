"""Critical-path split of MADPOSE_TIMELINE runs (engine.cpp Run::Timeline): per run,
time in main-thread launches, GPU waits, LO (prefix / steps), host decisions (exact /
resolve), sampler joins, draws, and the rest.  usage: python tools/timeline_summary.py LOG"""
import collections
import re
import sys

runs = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"\[timeline (\d+)\]\s+([\d.]+)\s+(\S+)\s+(-?\d+)", line)
    if m:
        runs[int(m.group(1))].append((float(m.group(2)), m.group(3), int(m.group(4))))
pairs = {"launch": "launched", "wait": "ready", "lo": "lo_end", "exact": "decided", "resolve": "decided",
         "join_sampler": "joined", "join_spec": "joined", "draw": None}
for r, ev in sorted(runs.items()):
    main = [e for e in ev if not e[1] in ("h2d", "solve_launched", "score_launched", "solve_us", "score_us")]
    acc = collections.Counter()
    gpu = collections.Counter()
    for e in ev:
        if e[1] in ("solve_us", "score_us"):
            gpu[e[1]] += e[2]
    for i, (t, what, a) in enumerate(main):
        if what in pairs and pairs[what]:
            for t2, w2, _ in main[i + 1:]:
                if w2 == pairs[what]:
                    acc[what] += t2 - t
                    break
        if what == "lo":
            for t2, w2, _ in main[i + 1:]:
                if w2 == "lo_prefix_end":
                    acc["lo_prefix"] += t2 - t
                    break
    total = main[-1][0]
    rest = total - sum(v for k, v in acc.items() if k != "lo_prefix")
    print(f"run {r}: total {total:.0f} us | " + " | ".join(f"{k} {v:.0f}" for k, v in acc.most_common()) +
          f" | other {rest:.0f} | device solve {gpu['solve_us']} score {gpu['score_us']}")
