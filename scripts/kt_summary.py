"""Per-kernel summary (calls, avg us, total ms) from a rocprofv3 rocpd database.
usage: python scripts/kt_summary.py DIR [N]"""
import glob
import sqlite3
import sys

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
c = sqlite3.connect(db)
q = ("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1e6 from kernels group by name "
     "order by sum(end-start) desc limit ?")
for name, cnt, avg, tot in c.execute(q, (n,)):
    print(f"{name[:72]:72s} {cnt:6d} {avg:9.2f} us {tot:9.3f} ms")
