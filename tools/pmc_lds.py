"""LDS bank conflicts per kernel of a C2 call (rocprofv3 --pmc CSV from tools/trace_c2.py run).

  rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES --output-format csv \
      -d gpurun_out/pmc_lds -o run -- python tools/trace_c2.py run
  python tools/pmc_lds.py gpurun_out/pmc_lds/run_counter_collection.csv
SQ_LDS_BANK_CONFLICT = extra LDS cycles from conflicts, SQ_LDS_IDX_ACTIVE = all LDS-array cycles
(MI355X_MICROARCH.md, LDS): conflict share = BANK_CONFLICT / IDX_ACTIVE.
"""
import csv
import statistics
import sys
from collections import defaultdict


def main(path):
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0][:80]
        per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, cs in sorted(per.items(), key=lambda kv: -statistics.median(kv[1].get("SQ_WAVE_CYCLES", [0]))):
        med = {k: statistics.median(v) for k, v in cs.items()}
        bc, act = med.get("SQ_LDS_BANK_CONFLICT", 0.0), med.get("SQ_LDS_IDX_ACTIVE", 0.0)
        share = bc / act if act else 0.0
        print(f"{name:80s} conflict {bc:12.0f} active {act:12.0f} share {share:6.3f} lds_insts "
              f"{med.get('SQ_INSTS_LDS', 0):10.0f} wave_cycles {med.get('SQ_WAVE_CYCLES', 0):12.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
