"""Per-kernel duration summary from a rocprofv3 rocpd database (kernel trace).
Usage: python tools/kstats.py DB [DB...] [--limit N] [--full] [--per-step K]
--full prints whole kernel names; --per-step K adds the per-step total (total / K)."""
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
limit = 40
full = "--full" in sys.argv
per_step = 0
if "--per-step" in sys.argv:
    per_step = int(sys.argv[sys.argv.index("--per-step") + 1])
    args = [a for a in args if a != str(per_step)]
if "--limit" in sys.argv:
    limit = int(sys.argv[sys.argv.index("--limit") + 1])
    args = [a for a in args if a != str(limit)]
for db in args:
    c = sqlite3.connect(db)
    q = f"""select name, count(*), avg(end-start)/1e6, min(end-start)/1e6, max(end-start)/1e6, sum(end-start)/1e6
           from kernels group by name order by sum(end-start) desc limit {limit}"""
    print(db)
    print(f'{"kernel":60s} {"n":>4} {"avg_ms":>10} {"min_ms":>10} {"max_ms":>10} {"total_ms":>10}')
    tot = 0.0
    for name, n, avg, mn, mx, t in c.execute(q):
        tot += t
        nm = name if full else f"{name[:60]:60s}"
        ps = f" {t / per_step:10.3f}" if per_step else ""
        print(f"{nm} {n:4d} {avg:10.3f} {mn:10.3f} {mx:10.3f} {t:10.3f}{ps}")
    n_all, t_all = c.execute("select count(*), sum(end-start)/1e6 from kernels").fetchone()
    print(f"all kernels: {n_all} dispatches, {t_all:.3f} ms")
