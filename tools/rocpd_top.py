"""Print the top kernels of a rocprofv3 rocpd database: python tools/rocpd_top.py gpurun_out/x/run_results.db [n]"""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
for name, calls, total, avg, pct in con.execute("select * from top_kernels limit ?", (n,)):
    print(f"{avg:10.3f} us avg  {calls:6d} calls  {pct:5.1f}%  {name[:110]}")
