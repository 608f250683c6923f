"""Per-dispatch PMC counters from a rocprofv3 SQLite output (pmc_results.db): one row per kernel dispatch with the
workgroup size, grid, duration and the summed counter values (instances summed).

Usage: python tools/pmc_db.py gpurun_out/<dir>/pmc_results.db [kernel-substring]
"""
import sqlite3
import sys
from collections import defaultdict


def dispatches(path, match=None):
    con = sqlite3.connect(path)
    names = {r[0]: r[1] for r in con.execute("select id, name from rocpd_info_pmc")}
    ksym = {r[0]: r[1] for r in con.execute("select id, display_name from rocpd_info_kernel_symbol")}
    rows = {}
    for (did, kid, ev, wg, grid, st, en) in con.execute(
            "select id, kernel_id, event_id, workgroup_size_x, grid_size_x, start, end from rocpd_kernel_dispatch"):
        name = ksym.get(kid, "?")
        if match and match not in name:
            continue
        rows[ev] = {"kernel": name, "wg": wg, "grid": grid, "ns": en - st, "pmc": defaultdict(float)}
    for (ev, pid, val) in con.execute("select event_id, pmc_id, value from rocpd_pmc_event"):
        if ev in rows:
            rows[ev]["pmc"][names.get(pid, str(pid))] += val
    return list(rows.values())


if __name__ == "__main__":
    for r in dispatches(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None):
        print(r["kernel"][:60], "wg", r["wg"], "grid", r["grid"], "us %.1f" % (r["ns"] / 1e3),
              " ".join(f"{k}={v:.4g}" for k, v in sorted(r["pmc"].items())))
