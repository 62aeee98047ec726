"""Summarise rocprofv3 PMC / kernel-trace databases (rocpd sqlite) per kernel: mean counter value
per dispatch and mean duration. Usage: python scripts/pmc_summary.py DB [DB ...] [--match SUBSTR]"""
import argparse
import re
import collections
import sqlite3


def short(name: str) -> str:
    if name.startswith("Custom_Cijk") or name.startswith("Cijk"):
        return "hipBLASLt " + name.split("_MT")[1].split("_")[0] if "_MT" in name else name[:60]
    base = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    return re.sub(r"^.*::", "", base.split("<")[0]) + ("<" + base.split("<", 1)[1] if "<" in base else "")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dbs", nargs="+")
    p.add_argument("--match", default="", help="only kernels whose name contains this")
    a = p.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for db in a.dbs:
        c = sqlite3.connect(db)
        names = [r[0] for r in c.execute("select name from sqlite_master")]
        if "counters_collection" in names:
            for kn, cn, v, vg, ag, sg, lds, scr, wg in c.execute(
                    "select kernel_name, counter_name, value, vgpr_count, accum_vgpr_count, "
                    "sgpr_count, lds_block_size, scratch_size, workgroup_size from counters_collection"):
                if a.match in kn:
                    vals[short(kn)][cn].append(v)
                    meta[short(kn)] = (vg, ag, sg, lds, scr, wg)
        for kn, dur in c.execute("select name, duration from kernels"):
            if a.match in kn:
                vals[short(kn)]["duration_us"].append(dur / 1e3)
    for k, cs in vals.items():
        print(f"== {k}  (vgpr, agpr, sgpr, lds, scratch, wg) = {meta.get(k)}")
        for cn in sorted(cs):
            v = cs[cn]
            print(f"   {cn:34s} mean {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
