"""Per-launch HBM bytes of one rank's shard (scripts/pmc_shard.sh output) merged into
profiles/pmc_traffic.json under "shards" -> "<config>/w<W>" -> kernel, so bench.py can
report roofline.traffic for an N > 1 line (rank 0's shard, measured on one GPU with
--emulate-world W: the same node range and kernels rank 0 runs).

  python scripts/pmc_shard_sum.py <traffic.json> <pmcshard dir>...
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


def main(traffic_json, dirs):
    t = json.load(open(traffic_json))
    shards = t.setdefault("shards", {})
    for d in dirs:
        m = re.search(r"pmcshard_([^_]+)_(C\d)_w(\d+)", os.path.basename(os.path.normpath(d)))
        tag, cfg, w = m.group(1), m.group(2), int(m.group(3))
        pmc = defaultdict(lambda: defaultdict(list))
        for f in glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv")):
            for row in csv.DictReader(open(f)):
                pmc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
        ent = {}
        for k, c in pmc.items():
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                fk = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
                wk = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
                ent[k] = {"hbm_bytes_per_launch": (2 * fk + wk) * 1024, "fetch_kib": fk, "write_kib": wk}
        shards[f"{cfg}/w{w}"] = {"source": f"pmcshard_{tag}", "kernels": ent}
        for k in ("reduce_kernel<2>", "reduce_kernel<2, false>", "reduce_kernel<2, true>",
                  "fit_kernel<false>", "fit_kernel<true>"):
            if k in ent:
                print(f"{cfg} w{w} {k}: {ent[k]['hbm_bytes_per_launch'] / 1e6:.2f} MB per launch")
    t["shards_method"] = ("rank 0's node shard of a W-way strong-scaling split, run alone on one "
                          "GPU (bench.py --emulate-world W), FETCH_SIZE / WRITE_SIZE in separate "
                          "passes; bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 per dispatch")
    json.dump(t, open(traffic_json, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
