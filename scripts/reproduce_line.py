"""Recompute the bench line's roofline figures from what profiles/<round>/ keeps.

    python scripts/reproduce_line.py BENCH_JSON BENCH_PMC_JSON KERNEL_TRACE_CSV [--warmup W --steps K] > repro.json

BENCH_JSON        the line bench.py printed (run with --pmc-keep DIR)
BENCH_PMC_JSON    DIR/bench_pmc.json: the per-dispatch rows of the line's own PMC passes (the same rows its
                  roofline averaged; pmc_summary_<round>.json is this file's summary)
KERNEL_TRACE_CSV  rocprofv3 --kernel-trace of the same bench command (--no-pmc --no-cpu-baseline --no-configs): its
                  FAST k_render launches split into the unordered first frame, the line's timed launches and the
                  later ordered ones (host-output frames)

Prints the figures recomputed from those files next to the line's own (roofline.frac = VALU issue, cache.l2_frac, latency.frac,
hbm.frac) and the kernel statistics of each launch group."""
import argparse
import csv
import json
import statistics
import sys

N_SIMD, N_XCD, HBM, L2 = 1024, 8, 8000.0, 34500.0


def trace_groups(path, warmup, steps):
    rows = [r for r in csv.DictReader(open(path)) if "k_render<false" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]

    def st(x):
        return {"launches": len(x), "avg_ms": round(statistics.mean(x), 4) if x else None,
                "min_ms": round(min(x), 4) if x else None, "max_ms": round(max(x), 4) if x else None}

    # launch 0: the first frame (supertile order, no previous costs); 1..warmup: ordered warm-up; then the timed K
    return {"first_frame": st(ms[:1]), "warmup": st(ms[1:1 + warmup]), "timed": st(ms[1 + warmup:1 + warmup + steps]),
            "later_ordered": st(ms[1 + warmup + steps:]), "all": st(ms)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bench")
    ap.add_argument("pmc")
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    line = json.loads([x for x in open(a.bench) if x.startswith("{")][-1])
    pmc = json.load(open(a.pmc))
    roof = line["roofline"]
    kms = roof["kernel_ms_avg"]
    # per-counter averages over the kept rows (each pass's timed dispatches of the frame's grid)
    acc = {}
    for r in pmc["rows"]:
        acc.setdefault(r["counter"], []).append(r["value"])
    avg = {k: sum(v) / len(v) for k, v in acc.items()}
    cyc = avg["GRBM_GUI_ACTIVE"] / N_XCD
    valu = 2.0 * avg["SQ_INSTS_VALU"] / (N_SIMD * cyc)
    traffic = avg["FETCH_SIZE"] * 1024 * 2 + avg["WRITE_SIZE"] * 1024
    hbm = traffic / (kms * 1e-3) / 1e9 / HBM
    gather = roof["reference_gather"]["bytes_per_launch"] / (kms * 1e-3) / 1e9
    l2 = avg["TCC_REQ_sum"] * 128.0 / (kms * 1e-3) / 1e9 / L2 if "TCC_REQ_sum" in avg else None
    lat = roof.get("latency", {})
    lat_frac = None
    if lat and "SQ_WAVE_CYCLES" in avg:
        life = 4.0 * avg["SQ_WAVE_CYCLES"] / avg["SQ_WAVES"]
        lat_frac = (lat["node_visits_per_wave"] + lat["leaf_visits_per_wave"]) * lat["l2_hit_latency_cycles"] / life
    out = {
        "line": {"roofline.bound": roof["bound"], "roofline.frac": roof["frac"],
                 "valu_issue_frac": roof.get("valu_issue_frac", roof["frac"] if roof["bound"] == "issue" else None),
                 "reference_gather.equivalent_gbs": roof["reference_gather"]["equivalent_gbs"],
                 "hbm.frac": roof["hbm"]["frac"], "cache.l2_frac": roof.get("cache", {}).get("l2_frac"),
                 "latency.frac": lat.get("frac"), "binding": roof.get("binding"), "kernel_ms_avg": kms,
                 "ms_per_step": line["ms_per_step"]},
        "recomputed": {"valu_issue_frac": round(valu, 4), "reference_gather.equivalent_gbs": round(gather, 1),
                       "hbm.frac": round(hbm, 5), "cache.l2_frac": None if l2 is None else round(l2, 4),
                       "latency.frac": None if lat_frac is None else round(lat_frac, 4),
                       "traffic_bytes_per_launch": traffic, "dispatches_per_pass": {
                           str(p): len({r["dispatch"] for r in pmc["rows"] if r["pass"] == p})
                           for p in sorted({r["pass"] for r in pmc["rows"]})}},
        "kernel_trace": trace_groups(a.trace, a.warmup, a.steps),
        "formulae": {"valu_issue_frac": "2 x SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)",
                     "reference_gather.equivalent_gbs": "SURVEY 8d bytes_per_launch / kernel_ms_avg (not a fraction)",
                     "cache.l2_frac": "TCC_REQ_sum x 128 B / kernel_ms_avg / 34.5 TB/s",
                     "latency.frac": "(node + leaf visits per wave) x 200 cycles / (4 x SQ_WAVE_CYCLES / SQ_WAVES)",
                     "hbm.frac": "(FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024) / kernel_ms_avg / 8 TB/s"},
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
