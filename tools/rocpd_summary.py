#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (--kernel-trace --stats run) as a kernel-stats CSV:
name, calls, total/avg/min/max duration (ns), share, plus per-kernel launch resources.

    python tools/rocpd_summary.py gpurun_out/<run>/prof/run_results.db > profiles/<name>.csv
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
                     "max(grid_x), max(workgroup_x), max(lds_size), max(scratch_size), max(vgpr_count), "
                     "max(sgpr_count) from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print("Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage,GridX,WorkgroupX,LdsBytes,ScratchBytes,"
          "VGPR,SGPR")
    for r in rows:
        print('"%s",%d,%d,%.1f,%d,%d,%.3f,%d,%d,%d,%d,%d,%d' % (r[0], r[1], r[2], r[3], r[4], r[5],
                                                                100.0 * r[2] / total, *r[6:]))


if __name__ == "__main__":
    main(sys.argv[1])
