"""Worker for tests/test_native_gpu.py: several ranks sharing ONE GPU over HIP IPC.

RCCL refuses two ranks on one device, so the control plane is gloo and only backend=ipc
configurations run here. Prints one JSON line: {label: "ok" | error}.
"""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.primitives.tp_columnwise.native import NativeTPColumnwise
    from ddlb_amd.primitives.tp_rowwise.native import NativeTPRowwise

    comm = Communicator()
    comm.ensure_process_group()
    cfgs = json.loads(os.environ["DDLB_TEST_CFGS"])
    res = {}
    only = os.environ.get("DDLB_TEST_ONLY", "")
    for label, prim, opts in cfgs:
        if only and only not in label:
            continue
        if os.environ.get("DDLB_TEST_PROGRESS"):
            print(f"[rank {comm.rank}] {label}", file=sys.stderr, flush=True)
        try:
            cls = NativeTPColumnwise if prim == "col" else NativeTPRowwise
            impl = cls(m=opts.pop("m", 1536), n=512, k=768, dtype=opts.pop("dtype", "bfloat16"),
                       **opts)
            for it in range(4):
                out = impl.run()
                torch.cuda.synchronize()
                impl.validate(out)
            for it in range(12):  # back-to-back epochs, no host sync in between (bench loop)
                out = impl.run()
            torch.cuda.synchronize()
            impl.validate(out)
            impl.close()
            res[label] = "ok"
        except Exception as e:  # report, keep going (all ranks run the same list)
            res[label] = f"{type(e).__name__}: {e}"[:400]
        comm.barrier()
    if comm.rank == 0:
        print("RESULT " + json.dumps(res), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
