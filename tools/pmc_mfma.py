"""Per-kernel MFMA utilisation from one rocprofv3 PMC pass.

Usage: python tools/pmc_mfma.py <counter_collection.csv> <kernel_trace.csv> [out.json [workload [command [commit]]]]

Counters (one pass: 3 SQ + 1 GRBM slots): SQ_VALU_MFMA_BUSY_CYCLES (cycles the matrix pipe is busy,
summed over every SIMD), SQ_INSTS_VALU_MFMA_MOPS_F32 (fp32 MFMA math ops / 512), SQ_BUSY_CU_CYCLES
and GRBM_GUI_ACTIVE (GPU busy cycles, summed over the 8 XCDs by rocprofv3 -- MI355X_MICROARCH.md
"DVFS give-back").  Per kernel (mean per dispatch):

  flop         = MOPS_F32 x 512                      (MfmaFlopsF32, counter_defs.yaml)
  mfma_busy    = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)   (MfmaUtil, gfx950 formula)
  clock_ghz    = GRBM_GUI_ACTIVE / 8 / duration      (reads high below ~0.3 ms dispatches)
  tflops_pmc   = flop / duration of the same (counter-collecting) dispatch

The durations of a counter-collecting run are serialized dispatches; ``tflops_pmc`` is therefore a
lower bound of the rate in the captured step (bench.py reports that rate from HIP events).
"""
import collections
import csv
import json
import sys

CTRS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_BUSY_CU_CYCLES", "GRBM_GUI_ACTIVE")
SIMDS = 256 * 4
XCDS = 8


def _name(s):
    return s.split("(")[0].replace("void ", "").strip()


def _key(row):
    """kernel name + grid size: one kernel template serves several GEMM shapes per step."""
    return f"{_name(row['Kernel_Name'])} grid={row['Grid_Size']}"


def summarise(ctr_csv):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))   # name -> dispatch -> counter
    dur = collections.defaultdict(dict)
    with open(ctr_csv, newline="") as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] not in CTRS:
                continue
            name = _key(row)
            d = int(row["Dispatch_Id"])
            per[name][d][row["Counter_Name"]] = per[name][d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            dur[name][d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    out = {}
    for name, ds in per.items():
        n = len(ds)
        mean = {c: sum(v.get(c, 0.0) for v in ds.values()) / n for c in CTRS}
        t = sum(dur[name].values()) / n
        gui = mean["GRBM_GUI_ACTIVE"] / XCDS
        flop = mean["SQ_INSTS_VALU_MFMA_MOPS_F32"] * 512.0
        out[name] = {"dispatches": n, "duration_s": t, "flop": flop,
                     "mfma_busy": mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * SIMDS) if gui else None,
                     "clock_ghz": gui / t / 1e9 if t > 0 else None,
                     "tflops_pmc": flop / t / 1e12 if t > 0 else None,
                     "counters": mean}
    return out


def _src_hash():
    """bench.kernel_src_hash(): which kernel sources these counters were recorded with."""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_src_hash
    return kernel_src_hash()


if __name__ == "__main__":
    res = summarise(sys.argv[1])
    doc = {"workload": sys.argv[4] if len(sys.argv) > 4 else "synth-20000",
           "command": sys.argv[5] if len(sys.argv) > 5 else None,
           "commit": sys.argv[6] if len(sys.argv) > 6 else None,
           "src_hash": _src_hash(),
           "formulas": {"flop": "SQ_INSTS_VALU_MFMA_MOPS_F32 * 512",
                        "mfma_busy": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)",
                        "clock_ghz": "GRBM_GUI_ACTIVE / 8 / duration"},
           "kernels": {k: v for k, v in res.items() if v["flop"] > 0}}
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(json.dumps(doc, indent=1) + "\n")
    for k, v in sorted(doc["kernels"].items(), key=lambda kv: -kv[1]["flop"] * kv[1]["dispatches"]):
        print(f"{k[:90]:90s} n={v['dispatches']:3d} GF={v['flop'] / 1e9:7.2f} t={v['duration_s'] * 1e6:7.1f}us "
              f"TF={v['tflops_pmc']:6.1f} busy={v['mfma_busy']:.3f} clk={v['clock_ghz']:.2f}")
