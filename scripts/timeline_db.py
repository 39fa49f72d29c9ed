"""Kernel timeline of the last bench step from a rocprofv3 rocpd database
(the default output format): start/end relative to the window's first kernel,
the gap to the previous kernel, the queue.
Usage: python scripts/timeline_db.py gpurun_out/prof/run_results.db [nkernels]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
nk = int(sys.argv[2]) if len(sys.argv) > 2 else 48
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
rows = db.execute("select * from kernels order by start").fetchall()
rows = [dict(zip(cols, r)) for r in rows][-nk:]
t0 = rows[0]["start"]
prev_end = t0
busy = 0
for r in rows:
    s, e = r["start"] - t0, r["end"] - t0
    gap = s - (prev_end - t0)
    prev_end = max(prev_end, r["end"])
    busy += e - s
    print(f"{s / 1000:8.1f} {e / 1000:8.1f} {(e - s) / 1000:6.1f} gap{gap / 1000:6.1f} "
          f"q{r.get('queue_id', r.get('stream_id', '?'))} {str(r['name'])[:48]:48s} "
          f"g={r.get('grid_x', r.get('grid_size_x', '?'))}")
print(f"span {(prev_end - t0) / 1000:.1f} us, kernel busy {busy / 1000:.1f} us")
