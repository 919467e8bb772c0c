#!/usr/bin/env python3
"""Summarise rocprofv3 output for profiles/.

  prof_summary.py stats <dir>          kernel_stats.csv -> markdown table, then per (kernel, grid)
  prof_summary.py pmc <dir> <counter>  counter_collection.csv -> per-kernel mean
  prof_summary.py calib <dir> <counter> <bytes>   counter / true bytes per calibration kernel
  prof_summary.py traffic <fetch_dir> <write_dir> <workload> <pixels> <alg_bytes_per_px>
                                       -> profiles/pmc_k1.json entry (HBM bytes per K1 launch)
  prof_summary.py traffic2 <fetch_dir> <write_dir> <workload> <pixels> <k1_alg_per_px> <k2_alg_per_px>
                                       -> pmc_k1.json entries <workload> (K1), <workload>_k2 (K2)
                                          and <workload>_two_launch (K1 + K2 of a frame), from
                                          the separate-launch passes (tools/k1_frames.py)
  prof_summary.py sq <out.json> <dir> [<dir> ...] -> K1 / K2 per-launch means of every counter
                                       in the passes, plus derived rates

FETCH_SIZE / WRITE_SIZE are KB per dispatch (rocprofv3 derived counters).
MI355X_MICROARCH.md (HBM): on gfx950 FETCH_SIZE reads half the bytes of a
wide coalesced stream, so the corrected read traffic is 2 x FETCH_SIZE; the
raw value is kept beside it because our gathers are not all 16-B streams.
"""
import csv
import glob
import json
import os
import statistics
import sys


def find(d, pattern):
    hits = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    if not hits:
        sys.exit(f"no {pattern} under {d}")
    return hits[0]


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    n = n.split("(")[0]
    for ns in ("bmfr::cols::", "bmfr::"):
        n = n.replace(ns, "")
    return n[:70]


def stats(d):
    rows = list(csv.DictReader(open(find(d, "*kernel_stats.csv"))))
    med = {}  # median duration per kernel from the kernel trace (steady state, without the cold first frames)
    hits = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if hits:
        for r in csv.DictReader(open(hits[0])):
            med.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = ["| kernel | calls | total ms | avg us | median us | min us | max us | % |",
           "|---|---|---|---|---|---|---|---|"]
    for r in rows:
        m = med.get(r["Name"])
        ms = f"{statistics.median(m) / 1e3:.1f}" if m else "-"
        out.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} | {ms} | {float(r['MinNs']) / 1e3:.1f} | "
                   f"{float(r['MaxNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    return "\n".join(out)


def by_grid(d):
    """Per (kernel, grid size): dispatches and mean / median duration from the
    kernel trace -- separates the image sizes one bench command runs."""
    rows = list(csv.DictReader(open(find(d, "*kernel_trace.csv"))))
    per = {}
    for r in rows:
        if not any(k in r["Kernel_Name"] for k in ("bmfr", "k_synth")):
            continue
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1))
        per.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = ["| kernel | work-groups | dispatches | mean us | median us |", "|---|---|---|---|---|"]
    for (k, g), v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        out.append(f"| {k} | {g} | {len(v)} | {statistics.mean(v):.1f} | {statistics.median(v):.1f} |")
    return "\n".join(out)


def pmc(d, counter):
    rows = list(csv.DictReader(open(find(d, "*counter_collection.csv"))))
    per = {}
    for r in rows:
        if r.get("Counter_Name", r.get("Counter-Name")) != counter:
            continue
        per.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in per.items()}


# K1 / K2 of the default configuration; K1_NAME / K2_NAME select another one
# (config 5: the mangled names "_ZN4bmfr4cols12k_fused_colsILi4ELi9EDF16_Lb0E" / "_ZN4bmfr11k_fused_taaIDF16_E").
KERNELS = {"K1 k_fused_cols": os.environ.get("K1_NAME", "k_fused_cols<4, 6, float, false>"),
           "K2 k_fused_taa": os.environ.get("K2_NAME", "k_fused_taa<float>")}


def sq(dirs):
    out = {}
    for key, name in KERNELS.items():
        c = {}
        for d in dirs:
            for r in csv.DictReader(open(find(d, "*counter_collection.csv"))):
                if short(r["Kernel_Name"]).startswith(name):
                    c.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        e = {k: round(statistics.mean(v), 3) for k, v in sorted(c.items())}
        if "SQ_INSTS_VALU" in e and "SQ_WAVES" in e:
            e["valu_instr_per_wave"] = round(e["SQ_INSTS_VALU"] / e["SQ_WAVES"], 3)
            e["valu_instr_per_simd"] = round(e["SQ_INSTS_VALU"] / 1024, 3)  # 256 CUs x 4 SIMDs
        if "SQ_WAIT_ANY" in e and "SQ_WAVE_CYCLES" in e:
            e["wait_any_frac_of_wave_cycles"] = round(e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"], 3)
        for k in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in e and "SQ_WAVE_CYCLES" in e:
                e[k.lower() + "_frac_of_wave_cycles"] = round(e[k] / e["SQ_WAVE_CYCLES"], 3)
        if "SQC_ICACHE_MISSES" in e and "SQC_ICACHE_HITS" in e:
            e["icache_miss_rate"] = round(e["SQC_ICACHE_MISSES"] / (e["SQC_ICACHE_MISSES"] + e["SQC_ICACHE_HITS"]), 4)
        if "GRBM_GUI_ACTIVE" in e:
            e["kernel_cycles_per_xcd"] = round(e["GRBM_GUI_ACTIVE"] / 8, 3)
            if "TA_BUSY_avr" in e:
                e["ta_busy_frac"] = round(e["TA_BUSY_avr"] / e["kernel_cycles_per_xcd"], 3)
        out[key] = e
    return out


def main():
    cmd = sys.argv[1]
    if cmd == "stats":
        print(stats(sys.argv[2]))
        print()
        print("Per work-group count (one bench command runs several image sizes):")
        print()
        print(by_grid(sys.argv[2]))
    elif cmd == "pmc":
        print(json.dumps(pmc(sys.argv[2], sys.argv[3]), indent=1))
    elif cmd == "calib":
        true_kb = int(sys.argv[4]) / 1024
        for k, v in pmc(sys.argv[2], sys.argv[3]).items():
            print(f"{k:40s} {sys.argv[3]} {v:12.0f} KB  counted/true {v / true_kb:.3f}")
    elif cmd == "sq":
        path = sys.argv[2]
        d = sq(sys.argv[3:])
        json.dump(d, open(path, "w"), indent=1)
        print(json.dumps(d, indent=1))
    elif cmd in ("traffic", "traffic2"):
        fetch_dir, write_dir, workload, px, alg = sys.argv[2:7]
        fetch, write = pmc(fetch_dir, "FETCH_SIZE"), pmc(write_dir, "WRITE_SIZE")

        def entry(name, alg_bytes):
            f = next(v for k, v in fetch.items() if k.startswith(name))
            w = next(v for k, v in write.items() if k.startswith(name))
            return {"fetch_kb_raw": f, "write_kb": w,
                    "hbm_bytes_per_launch": (2 * f + w) * 1024,
                    "hbm_bytes_per_launch_raw": (f + w) * 1024,
                    "algorithmic_bytes_per_launch": alg_bytes,
                    "note": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE half-count correction, "
                            "MI355X_MICROARCH.md HBM); raw = FETCH_SIZE + WRITE_SIZE"}
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_k1.json")
        d = json.load(open(path)) if os.path.exists(path) else {}
        new = {workload: entry(os.environ.get("K1_NAME", "k_fused_cols<4, 6"), int(px) * int(alg))}
        if cmd == "traffic2":
            k1, k2 = new[workload], entry(os.environ.get("K2_NAME", "k_fused_taa<float>"), int(px) * int(sys.argv[7]))
            new[workload + "_k2"] = k2
            new[workload + "_two_launch"] = {
                k: k1[k] + k2[k] for k in ("fetch_kb_raw", "write_kb", "hbm_bytes_per_launch",
                                           "hbm_bytes_per_launch_raw", "algorithmic_bytes_per_launch")}
            new[workload + "_two_launch"]["note"] = "K1 + K2 launches of one frame (the 4K frames' form); " + k1["note"]
        d.update(new)
        json.dump(d, open(path, "w"), indent=1)
        print(json.dumps(new, indent=1))


if __name__ == "__main__":
    main()
