"""Summarise a tools/profile.sh run into profiles/<tag>_<config>.md and profiles/traffic_<config>.json.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KB; on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so it is doubled.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("k_blkp_ichain", "k_blkp_phase", "k_terminal_cost", "k_blkp_exp", "k_blkp_dual", "k_blkp_chain", "k_blkp_int", "k_minmax", "k_blkseg_fwd", "k_blkseg_bwd", "k_blkp_grad", "k_blkseg_eval", "k_zero_rows", "k_bgemm_glds", "k_form_norm2", "k_blku_rec", "k_blku_fwd", "k_blku_bwdg", "k_blku_bwd", "k_blku_grad", "k_blku_dual", "k_blkrot_dual", "k_blkrot_fwd", "k_blkrot_bwd", "k_blk_dual", "k_blk_grad", "k_blk_fwd", "k_blk_bwd", "k_tchain_mf_dual", "k_grad_rr_c", "k_spec_bound", "k_tchain_mf_fwd", "k_tchain_mf_bwd", "k_tchain_prep", "k_tchain_fwd", "k_tchain_bwd", "k_pade_units",
           "k_argmin_seed", "k_expm_rr_ps", "k_expm_rr_mix", "k_expm_rr", "k_expm", "k_chain_fwd", "k_chain_bwd", "k_grad_rr_q", "k_grad_rr_p", "k_grad_rr_s", "k_grad", "k_bgemm", "k_form_norm", "k_lincomb", "k_gen_contract")


def short(name, variants=False):
    if "k_blkseg_eval<" in name:  # the split call form's halves: template argument MODE (qoc_blkseg.hpp)
        args = name.split("k_blkseg_eval<", 1)[1].split(">", 1)[0].split(",")
        mode = int(args[3]) if len(args) >= 4 and args[3].strip().isdigit() else 0
        return {1: "k_blkseg_fwd", 2: "k_blkseg_bwd"}.get(mode, "k_blkseg_eval")
    if variants and "k_bgemm<" in name:
        return "k_bgemm<" + name.split("k_bgemm<", 1)[1].split(">", 1)[0] + ">"
    for k in KERNELS:
        if k in name:
            return k
    return name.split("(")[0][:60]


def stats(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    rows = []
    if f:
        for r in csv.DictReader(open(f[0])):
            rows.append(r)
    return rows, (f[0] if f else None)


def pmc(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(list))
    if not f:
        return acc
    for r in csv.DictReader(open(f[0])):
        acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main(out_dir, cfg, tag, repo=".", form=""):
    form = f" --call-form {form}" if form else ""
    rows, src = stats(os.path.join(out_dir, "trace"))
    fetch = pmc(os.path.join(out_dir, "pmc_fetch"))
    write = pmc(os.path.join(out_dir, "pmc_write"))
    sq = pmc(os.path.join(out_dir, "pmc_sq"))
    for k, v in pmc(os.path.join(out_dir, "pmc_sq2")).items():  # second SQ pass (wait / busy cycles)
        sq.setdefault(k, {}).update(v)
    lines = [f"# rocprofv3 summary — {tag}, config `{cfg}`", "",
             f"Source: `{src}` (kernel-trace --stats of `bench.py --config {cfg} --warmup 1 --no-cpu{form}` (tools/profile*.sh)).", "",
             "| kernel | calls | avg ms | total ms | % |", "|---|---|---|---|---|"]
    for r in rows:
        name = short(r.get("Name", r.get("KernelName", "")), variants=True)
        calls = r.get("Calls", "")
        avg = float(r.get("AverageNs", 0)) / 1e6
        tot = float(r.get("TotalDurationNs", 0)) / 1e6
        pct = r.get("Percentage", "")
        lines.append(f"| {name} | {calls} | {avg:.3f} | {tot:.2f} | {pct} |")
    traffic = {}
    lines += ["", "HBM traffic per launch from PMC (separate passes; FETCH_SIZE doubled per gfx950 rule):", "",
              "| kernel | FETCH_SIZE KB (raw, mean) | WRITE_SIZE KB (mean) | HBM bytes/launch (corrected) |",
              "|---|---|---|---|"]
    for k in KERNELS:
        fe = fetch.get(k, {}).get("FETCH_SIZE", [])
        wr = write.get(k, {}).get("WRITE_SIZE", [])
        if not fe and not wr:
            continue
        fm = sum(fe) / len(fe) if fe else 0.0
        wm = sum(wr) / len(wr) if wr else 0.0
        b = (2 * fm + wm) * 1024.0
        traffic[k] = b
        lines.append(f"| {k} | {fm:.0f} | {wm:.0f} | {b / 1e9:.3f} GB |")
    if sq:
        names = sorted({n for c in sq.values() for n in c})
        lines += ["", "SQ counters (mean per launch):", "", "| kernel | " + " | ".join(names) + " |",
                  "|---|" + "---|" * len(names)]
        for k in KERNELS:
            c = sq.get(k)
            if c:
                m = {n: (sum(v) / len(v)) for n, v in c.items()}
                lines.append(f"| {k} | " + " | ".join(f"{m.get(n, 0):.3g}" for n in names) + " |")
    os.makedirs(os.path.join(repo, "profiles"), exist_ok=True)
    suffix = "_" + form.split()[-1] if form else ""
    open(os.path.join(repo, "profiles", f"{tag}_{cfg}{suffix}.md"), "w").write("\n".join(lines) + "\n")
    if traffic:  # labelled with where the bytes came from (bench.py copies the label into roofline.traffic_source)
        json.dump({"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, FETCH doubled) of "
                             f"bench.py --config {cfg} --warmup 1 --no-cpu{form}", "run": tag,
                   "counters": ["FETCH_SIZE", "WRITE_SIZE"], "kernels": traffic},
                  open(os.path.join(repo, "profiles", f"traffic_{cfg}{suffix}.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], form=sys.argv[4] if len(sys.argv) > 4 else "")
