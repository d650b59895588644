"""Summarise a scripts/profile.sh output dir into a markdown table (profiles/).

Per kernel: calls and average duration (kernel trace), and per-dispatch averages of
every PMC counter collected in the separate passes.  FETCH_SIZE/WRITE_SIZE are in
KiB; HBM bytes apply the gfx950 correction of MI355X_MICROARCH.md §HBM
(FETCH_SIZE reads 1/2 of wide coalesced streaming reads -> x2).
Derived columns: clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; VALU issue = wave64 VALU
instructions x 4 cycles / (1024 SIMDs x duration x clock).

  python scripts/summarize_prof.py <profile dir> <out.md> [<traffic.json>]

The optional JSON holds the per-launch HBM traffic per kernel; bench.py reports it as
roofline.traffic (profiles/pmc_traffic.json).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("kcc::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)


def main(d, out=None, traffic_json=None):
    stats = {}
    for row in csv.DictReader(open(glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))[0])):
        stats[short(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]),
                                     float(row["Percentage"]))
    pmc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            pmc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    lines = ["| kernel | calls | avg us | % time | " + " | ".join(
        ["FETCH_SIZE KiB", "WRITE_SIZE KiB", "HBM MB (2xF+W)", "SQ_INSTS_VALU", "SQ_WAVES",
         "clock GHz", "VALU issue %"]) + " |", "|" + "---|" * 11]
    traffic = {}
    for k, (calls, avg, pct) in sorted(stats.items(), key=lambda kv: -kv[1][2]):
        p = {c: sum(v) / len(v) for c, v in pmc.get(k, {}).items()}
        f, w = p.get("FETCH_SIZE"), p.get("WRITE_SIZE")
        hbm = (2 * f + w) * 1024 / 1e6 if f is not None and w is not None else None
        clk = issue = None
        if p.get("GRBM_GUI_ACTIVE"):
            clk = p["GRBM_GUI_ACTIVE"] / 8 / avg  # cycles per ns = GHz
            if p.get("SQ_INSTS_VALU"):
                issue = 100 * p["SQ_INSTS_VALU"] * 4 / (1024 * avg * clk)
        fmt = lambda x, s="{:.4g}": "-" if x is None else s.format(x)  # noqa: E731
        lines.append(f"| {k} | {calls} | {avg / 1e3:.2f} | {pct:.1f} | {fmt(f)} | {fmt(w)} | "
                     f"{fmt(hbm)} | {fmt(p.get('SQ_INSTS_VALU'))} | {fmt(p.get('SQ_WAVES'))} | "
                     f"{fmt(clk, '{:.3f}')} | {fmt(issue, '{:.1f}')} |")
        if hbm is not None:
            traffic[k] = {"hbm_bytes_per_launch": hbm * 1e6, "fetch_kib": f, "write_kib": w,
                          "avg_us": avg / 1e3, "clock_ghz": clk, "valu_issue_pct": issue}
    # read requests by size (TCC_EA0_RDREQ_{32B,64B,128B}, when a pass collected them): the
    # bytes the L2s asked the fabric for, a cross-check of the 2 x FETCH_SIZE correction
    sized = [(k, p) for k, p in ((k, {c: sum(v) / len(v) for c, v in pmc[k].items()}) for k in pmc)
             if "TCC_EA0_RDREQ_128B_sum" in p]
    if sized:
        lines += ["", "| kernel | RDREQ | 32B | 64B | 128B | read MB by size (32/64/128 B) | 2 x FETCH MB |",
                  "|---|---|---|---|---|---|---|"]
        for k, p in sized:
            n32, n64, n128 = (p.get(f"TCC_EA0_RDREQ_{b}B_sum", 0.0) for b in (32, 64, 128))
            mb = (32 * n32 + 64 * n64 + 128 * n128) / 1e6
            f = p.get("FETCH_SIZE")
            lines.append(f"| {k} | {p.get('TCC_EA0_RDREQ_sum', 0):.4g} | {n32:.4g} | {n64:.4g} | "
                         f"{n128:.4g} | {mb:.4g} | {'-' if f is None else f'{2 * f * 1024 / 1e6:.4g}'} |")
            if k in traffic:
                traffic[k]["read_bytes_by_req_size"] = mb * 1e6
    extra = ["", "Raw per-dispatch counter averages:", ""]
    for k in sorted(pmc):
        extra.append(f"- {k}: " + ", ".join(f"{c}={sum(v) / len(v):.6g}"
                                           for c, v in sorted(pmc[k].items())))
    text = "\n".join(lines + extra) + "\n"
    if out:
        open(out, "w").write(text)
    if traffic_json:
        keep = {}
        if os.path.exists(traffic_json):  # the shards' entries (scripts/pmc_shard_sum.py) stay
            old = json.load(open(traffic_json))
            keep = {k: old[k] for k in ("shards", "shards_method") if k in old}
        json.dump({**keep, "source": os.path.basename(os.path.normpath(d)),
                   "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes of "
                             "`python3 bench.py --no-cpu-baseline`; bytes = (2 x FETCH_SIZE + "
                             "WRITE_SIZE) x 1024 per dispatch (gfx950 FETCH_SIZE correction)",
                   "kernels": traffic}, open(traffic_json, "w"), indent=1)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None,
         sys.argv[3] if len(sys.argv) > 3 else None)
