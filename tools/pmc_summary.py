"""Summarize the separate rocprofv3 --pmc passes of tools/pmc.sh.

Per kernel: dispatches, mean FETCH_SIZE / WRITE_SIZE per dispatch (KB as
rocprofv3 reports them) and HBM bytes per dispatch, corrected as
MI355X_MICROARCH.md §HBM prescribes for gfx950 (FETCH_SIZE counts half of the
bytes of a wide coalesced read: x2; WRITE_SIZE exact).  From the SQ passes
(pmc3: instruction mix + SQ_WAVE_CYCLES / SQ_BUSY_CYCLES; pmc4: the disjoint
wait / issue-stall / active split) the per-dispatch means and the fractions
of wave time parked on memory (SQ_WAIT_ANY), stalled at issue
(SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY); SQ cycle counters count
quad-cycles (MI355X_MICROARCH.md PMC table).  Writes the table to
<out>/pmc_summary.json and the fill kernel's bytes per launch to
profiles/fill_traffic.json, which bench.py reports as roofline.traffic.

    python tools/pmc_summary.py gpurun_out profiles/r01 C3
    python tools/pmc_summary.py gpurun_out profiles/r04 C3J _c3j   (tools/pmc.sh _c3j passes;
        writes pmc_summary_c3j.json, fill_traffic.json only for C3)
"""
import csv
import json
import os
import sys
from collections import defaultdict


def read(path, counter):
    per = defaultdict(list)
    if not os.path.exists(path):
        return per
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            per[name].append(float(row["Counter_Value"]))
    return per


def main():
    src, out, config = sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "C3"
    tag = sys.argv[4] if len(sys.argv) > 4 else ""
    fetch = read(os.path.join(src, "pmc1" + tag, "p_counter_collection.csv"), "FETCH_SIZE")
    write = read(os.path.join(src, "pmc2" + tag, "p_counter_collection.csv"), "WRITE_SIZE")
    table = {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch[k]) / len(fetch[k]) if fetch[k] else 0.0
        w = sum(write[k]) / len(write[k]) if write[k] else 0.0
        table[k] = {"dispatches": max(len(fetch[k]), len(write[k])), "fetch_kb": round(f, 1), "write_kb": round(w, 1),
                    "hbm_bytes": int((2 * f + w) * 1024)}
    sq = {}
    for sub, names in (("pmc3", ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                                  "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"]),
                       ("pmc4", ["SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE"])):
        for cn in names:
            for k, v in read(os.path.join(src, sub + tag, "p_counter_collection.csv"), cn).items():
                sq.setdefault(k, {})[cn] = sum(v) / len(v)
    for k, d in sq.items():
        row = table.setdefault(k, {})
        row["sq"] = {cn: round(v, 1) for cn, v in d.items()}
        waves = d.get("SQ_WAVES") or 0
        if waves:
            row["per_wave"] = {cn.replace("SQ_INSTS_", "").lower(): round(d[cn] / waves, 1)
                               for cn in d if cn.startswith("SQ_INSTS_")}
            if "SQ_WAVE_CYCLES" in d:
                row["per_wave"]["wave_cycles"] = round(4 * d["SQ_WAVE_CYCLES"] / waves, 1)
        tot = sum(d.get(c, 0) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"))
        if tot:
            row["wave_time_split"] = {"wait_any": round(d.get("SQ_WAIT_ANY", 0) / tot, 3),
                                      "wait_inst_any": round(d.get("SQ_WAIT_INST_ANY", 0) / tot, 3),
                                      "active_inst_any": round(d.get("SQ_ACTIVE_INST_ANY", 0) / tot, 3)}
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "pmc_summary%s.json" % tag), "w") as fh:
        json.dump(table, fh, indent=1)
    fills = [k for k in table if k.startswith("ktas::fill_leaves") or k.startswith("ktas::fill_pair")]
    if fills and config == "C3":
        k = max(fills, key=lambda x: table[x]["dispatches"])
        doc = {"config": config, "kernel": k, "fill_bytes_per_launch": table[k]["hbm_bytes"],
               "fetch_kb": table[k]["fetch_kb"], "write_kb": table[k]["write_kb"],
               "correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950, MI355X_MICROARCH.md HBM section)",
               "source": os.path.join(out, "pmc_summary.json")}
        with open(os.path.join(os.path.dirname(out.rstrip("/")) or ".", "fill_traffic.json"), "w") as fh:
            json.dump(doc, fh, indent=1)
    print(json.dumps(table, indent=1))


if __name__ == "__main__":
    main()
