"""Per-kernel duration summary from a rocprofv3 SQLite results database
(rocprofv3 writes `<name>_results.db` by default): name, calls, average and
total microseconds, sorted by total -- the same columns as the CSV
`--stats` summary.  Usage: python tools/kstats_db.py <results.db> [N]"""

import sqlite3
import sys


def kernel_stats(db: str):
    c = sqlite3.connect(db)
    rows = c.execute(
        'select s.kernel_name, count(*), avg(d.end - d.start), sum(d.end - d.start) '
        'from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id '
        'group by s.kernel_name order by 4 desc').fetchall()
    return [(n, k, a / 1e3, t / 1e3) for n, k, a, t in rows]


if __name__ == '__main__':
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    for name, calls, avg_us, tot_us in kernel_stats(sys.argv[1])[:n]:
        print(f'{tot_us:12.1f} us {calls:6d} x {avg_us:10.2f} us  {name[:100]}')
