"""Per-kernel duration summary from a rocprofv3 rocpd SQLite database (rocprofv3 7.2's
default output): python tools/rocpd_stats.py <results.db> [name-filter]."""
import glob
import sqlite3
import sys


def stats(db, pat=""):
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    cols = [r[1] for r in c.execute(f"pragma table_info({ks})")]
    namecol = "kernel_name" if "kernel_name" in cols else ("display_name" if "display_name" in cols else "name")
    rows = c.execute(f"select s.{namecol}, d.end - d.start from {kd} d join {ks} s on d.kernel_id = s.id").fetchall()
    agg = {}
    for n, dur in rows:
        if pat and pat not in n:
            continue
        a = agg.setdefault(n, [0, 0.0])
        a[0] += 1
        a[1] += dur
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for _, v in out)
    print(f"{'calls':>6} {'total_ms':>10} {'avg_us':>9} {'pct':>5}  kernel")
    for n, (k, t) in out:
        print(f"{k:6d} {t / 1e6:10.3f} {t / k / 1e3:9.2f} {100 * t / tot:5.1f}  {n[:150]}")


if __name__ == "__main__":
    for db in glob.glob(sys.argv[1]) if "*" in sys.argv[1] else [sys.argv[1]]:
        stats(db, sys.argv[2] if len(sys.argv) > 2 else "")
