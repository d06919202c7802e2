"""Per-kernel duration summary from a rocprofv3 rocpd database (kernel trace)."""
import sqlite3
import sys

for db in sys.argv[1:]:
    c = sqlite3.connect(db)
    q = """select name, count(*), avg(end-start)/1e6, min(end-start)/1e6, max(end-start)/1e6, sum(end-start)/1e6
           from kernels group by name order by sum(end-start) desc limit 12"""
    print(db)
    print(f'{"kernel":60s} {"n":>4} {"avg_ms":>10} {"min_ms":>10} {"max_ms":>10} {"total_ms":>10}')
    for name, n, avg, mn, mx, tot in c.execute(q):
        print(f"{name[:60]:60s} {n:4d} {avg:10.3f} {mn:10.3f} {mx:10.3f} {tot:10.3f}")
