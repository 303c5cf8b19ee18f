"""Per-kernel summary of a rocprofv3 rocpd database (kernel trace): total/avg time and grid."""
import sqlite3
import sys

db = sys.argv[1]
runs = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
c = sqlite3.connect(db)
rows = c.execute("select name, grid_x, grid_y, workgroup_x, count(*), sum(end-start)/1e6, avg(end-start)/1e3 "
                 "from kernels group by name, grid_x, grid_y order by 6 desc limit 40").fetchall()
print("total_ms_per_run,calls,avg_us,grid_x,grid_y,wg,name")
for name, gx, gy, wg, n, tot, avg in rows:
    print(f"{tot / runs:.3f},{n},{avg:.1f},{gx},{gy},{wg},{name[:120]}")
