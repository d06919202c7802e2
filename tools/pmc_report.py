"""Summarise tools/pmc.sh output: per-kernel counter values per dispatch."""
import glob
import sqlite3
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(dict)
for db in sorted(glob.glob(f"{root}/p*/run_results.db")):
    c = sqlite3.connect(db)
    q = ("select kernel_name, counter_name, sum(value), count(distinct dispatch_id) from counters_collection "
         "group by kernel_name, counter_name")
    for k, cn, v, nd in c.execute(q):
        vals[k][cn] = v / max(nd, 1)
for k, d in sorted(vals.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if not any(s in k for s in ("route", "emit", "expand", "finish")):
        continue
    print(k[:70])
    w = d.get("SQ_WAVE_CYCLES")
    if w:
        print("   wave-cycle split: active %.0f%%  parked(waitcnt/barrier) %.0f%%  issue-stall %.0f%%" % (
            100 * d["SQ_ACTIVE_INST_ANY"] / w, 100 * d["SQ_WAIT_ANY"] / w, 100 * d["SQ_WAIT_INST_ANY"] / w))
    for cn in sorted(d):
        print(f"   {cn:22s} {d[cn]:.4g}")
