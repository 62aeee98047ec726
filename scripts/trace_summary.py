"""Per-stage summary of a rocprofv3 trace of a native plan run with ``trace=True``.

The executor wraps every op's enqueue in a roctx range named by ``Plan.labels()``; rocprofv3
(``--marker-trace --kernel-trace``) attributes each kernel dispatch to the range it was enqueued in
(``kernels.region``). This prints, per stage name, the kernels it launched, their count and mean
GPU time, plus the host time of the ranges themselves and the copy-engine transfers.

    python scripts/trace_summary.py gpurun_out/r3_6/trace_r0/tr_results.db
"""
import argparse
import collections
import json
import sqlite3


def main():
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("dbs", nargs="+")
    a = p.parse_args()
    for db in a.dbs:
        c = sqlite3.connect(db)
        print(f"== {db}")
        k = collections.defaultdict(list)
        for region, name, dur in c.execute("select region, name, duration from kernels"):
            if region:
                short = name.replace("void ", "").replace("(anonymous namespace)::", "")
                short = short.split("(")[0].split("<")[0].split("::")[-1]
                k[(region, short)].append(dur / 1e3)
        print("  GPU kernels per plan stage (roctx range of the enqueue):")
        for (region, short), d in sorted(k.items()):
            print(f"    {region:28s} {short:34s} n={len(d):4d} mean {sum(d) / len(d):9.1f} us")
        h = collections.defaultdict(list)
        for ext, dur in c.execute("select extdata, duration from regions"):
            try:
                msg = json.loads(ext).get("message", "?")
            except Exception:
                msg = "?"
            h[msg].append(dur / 1e3)
        print("  host enqueue time per stage (roctx range):")
        for msg, d in sorted(h.items()):
            print(f"    {msg:28s} n={len(d):4d} mean {sum(d) / len(d):9.1f} us")
        cp = [(sz, dur / 1e3) for sz, dur in c.execute("select size, duration from memory_copies")]
        if cp:
            tot = sum(s for s, _ in cp)
            print(f"  copy-engine transfers: n={len(cp)} total {tot / 2**20:.1f} MiB, mean "
                  f"{sum(d for _, d in cp) / len(cp):.1f} us, "
                  f"{tot / max(sum(d for _, d in cp), 1e-9) / 1e3:.1f} GB/s per copy (mean)")


if __name__ == "__main__":
    main()
