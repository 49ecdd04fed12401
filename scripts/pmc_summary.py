"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv) for k_render."""
import csv, glob, collections, json, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(float); cnt = collections.Counter(); meta = {}
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        if "k_render" not in row.get("Kernel_Name", ""): continue
        agg[row["Counter_Name"]] += float(row["Counter_Value"]); cnt[row["Counter_Name"]] += 1
        meta = {k: row[k] for k in ("Kernel_Name", "VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Grid_Size")}
avg = {k: agg[k] / cnt[k] for k in agg}
waves = avg.get("SQ_WAVES", 1)
out = {"meta": meta, "per_dispatch": avg,
       "per_wave": {k: avg[k] / waves for k in avg if k.startswith("SQ_INSTS")}}
if "GRBM_GUI_ACTIVE" in avg:
    out["gpu_cycles"] = avg["GRBM_GUI_ACTIVE"] / 8
if "SQ_WAVE_CYCLES" in avg:
    wc = avg["SQ_WAVE_CYCLES"]
    out["frac_of_wave_cycles"] = {k: avg[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                         "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS") if k in avg}
if "GRBM_GUI_ACTIVE" in avg and "SQ_INSTS_VALU" in avg:
    # the bench line's roofline (bound "issue"): 2 x VALU wave-instructions / (1024 SIMDs x the dispatch's cycles)
    out["valu_issue_frac"] = 2 * avg["SQ_INSTS_VALU"] / (1024 * out["gpu_cycles"])
if "FETCH_SIZE" in avg:
    out["hbm_read_bytes_per_dispatch_x2_corrected"] = avg["FETCH_SIZE"] * 1024 * 2
if "WRITE_SIZE" in avg:
    out["hbm_write_bytes_per_dispatch"] = avg["WRITE_SIZE"] * 1024
print(json.dumps(out, indent=1))
