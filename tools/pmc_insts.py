"""Per-kernel instruction counts per output point from tools/pmc_insts.sh's rocprofv3 passes.

SQ_INSTS_* count wave-instructions (one per wave per instruction issued); a wave covers 64 lanes x VEC
points per row (2D) / plane-row (3D), so "per 64 points" = count / (points / 64) is the instructions one
wave issues per lane-point.  SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_WAIT_* are quad-cycles per the MI355X guide.
Usage: python tools/pmc_insts.py gpurun_out/pmc_insts > profiles/r04/pmc_insts.txt
"""
import collections
import csv
import glob
import os
import re
import sys

# points per launch of each workload (interior points of the grid the bench solves)
POINTS = {"bratu2d": 4096 ** 2, "heat2d": 8192 ** 2, "heat2d_trapezoid_periodic": 8192 ** 2,
          "heat3d_midpoint": 512 ** 3, "heat3d_slab": 512 * 512 * 64,
          "heat3d_block": 256 ** 3}


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*", "", name).strip()
    return name.replace("nk::", "")


def load(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main(root):
    tags = sorted({os.path.basename(p).rsplit("_", 1)[0] for p in glob.glob(os.path.join(root, "*_[ABC]")) if os.path.isdir(p)})
    for tag in tags:
        n = POINTS.get(tag)
        data = collections.defaultdict(dict)
        for p in "ABC":
            d = os.path.join(root, f"{tag}_{p}")
            if not os.path.isdir(d):
                continue
            for k, ctrs in load(d).items():
                for c, v in ctrs.items():
                    data[k][c] = sum(v) / len(v)  # mean per launch
        print(f"== {tag} ({n} points per launch)")
        rows = []
        for k, c in data.items():
            if "SQ_WAVES" not in c or not n:
                continue
            if not k.startswith(("k_st", "k_mgs", "k_update")):
                continue
            per = n / 64.0  # wave-lane groups
            rows.append((c.get("SQ_WAVE_CYCLES", 0), k, c, per))
        for _, k, c, per in sorted(rows, reverse=True)[:12]:
            def g(name):
                return c.get(name, float("nan")) / per
            print(f"  {k[:64]:64s} waves {c['SQ_WAVES']:8.0f}  per 64 pts: VALU {g('SQ_INSTS_VALU'):6.1f} "
                  f"VMEM_RD {g('SQ_INSTS_VMEM_RD'):5.2f} VMEM_WR {g('SQ_INSTS_VMEM_WR'):5.2f} LDS {g('SQ_INSTS_LDS'):5.2f} "
                  f"SALU {g('SQ_INSTS_SALU'):5.1f} SMEM {g('SQ_INSTS_SMEM'):5.2f}")
            extra = []
            for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                         "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"):
                if name in c:
                    extra.append(f"{name[3:]} {c[name] / max(1.0, c.get('SQ_WAVE_CYCLES', 1.0)):.3f}")
            if extra:
                print("      (fractions of WAVE_CYCLES) " + "  ".join(extra))
            f64 = [x for x in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                               "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64",
                               "SQ_INSTS_VALU_CVT") if x in c]
            if f64:
                print("      per 64 pts: " + "  ".join(f"{x[14:]} {g(x):.1f}" for x in f64))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_insts")
