"""Summarise a scripts/profile.sh output dir into a markdown table (profiles/).

Per kernel: calls and average duration (kernel trace), and per-dispatch averages of
every PMC counter collected in the separate passes.  FETCH_SIZE/WRITE_SIZE are in
KiB; HBM bytes apply the gfx950 correction of MI355X_MICROARCH.md §HBM
(FETCH_SIZE reads 1/2 of wide coalesced streaming reads -> x2).
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("kcc::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)


def main(d, out=None):
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
         "VALU busy %", "GRBM_GUI_ACTIVE"]) + " |", "|" + "---|" * 11]
    for k, (calls, avg, pct) in sorted(stats.items(), key=lambda kv: -kv[1][2]):
        p = {c: sum(v) / len(v) for c, v in pmc.get(k, {}).items()}
        f, w = p.get("FETCH_SIZE"), p.get("WRITE_SIZE")
        hbm = (2 * f + w) * 1024 / 1e6 if f is not None and w is not None else None
        busy = None
        if p.get("SQ_ACTIVE_INST_VALU") and p.get("SQ_BUSY_CYCLES"):
            busy = 100 * p["SQ_ACTIVE_INST_VALU"] / max(p["SQ_BUSY_CYCLES"], 1)
        fmt = lambda x, s="{:.4g}": "-" if x is None else s.format(x)  # noqa: E731
        lines.append(f"| {k} | {calls} | {avg / 1e3:.2f} | {pct:.1f} | {fmt(f)} | {fmt(w)} | "
                     f"{fmt(hbm)} | {fmt(p.get('SQ_INSTS_VALU'))} | {fmt(p.get('SQ_WAVES'))} | "
                     f"{fmt(busy)} | {fmt(p.get('GRBM_GUI_ACTIVE'))} |")
    extra = ["", "Raw per-dispatch counter averages:", ""]
    for k in sorted(pmc):
        extra.append(f"- {k}: " + ", ".join(f"{c}={sum(v) / len(v):.6g}"
                                           for c, v in sorted(pmc[k].items())))
    text = "\n".join(lines + extra) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
