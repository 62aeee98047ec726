"""Which device work do the plan's signal / wait ops create? Run under
``rocprofv3 --kernel-trace`` to see whether hipStreamWriteValue32 / hipStreamWaitValue32 (and the
kernel-method signals) dispatch kernels — a kernel needs a free CU, so behind a GEMM that fills
the chip it cannot start until a workgroup retires."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from ddlb_amd.communicator import Communicator
    from ddlb_amd.parallel.context import NativeContext
    from ddlb_amd.parallel.plan import SIG_KERNEL, SIG_STREAM, Plan

    comm = Communicator()
    comm.ensure_process_group()
    ctx = NativeContext(comm)
    for method, tag in ((SIG_STREAM, "stream"), (SIG_KERNEL, "kernel")):
        plan = Plan(0, 1, nstreams=2, stream_priority=[0, 1])
        flags = plan.buffer("flags", 256, symmetric=True, zero=True)
        plan.signal(1, [flags], method=method)
        plan.wait_signal(0, [flags], method=method)
        bound = ctx.bind(plan)
        for _ in range(20):
            bound.run()
        torch.cuda.synchronize()
        bound.check_health()
        print(f"{tag}: 20 signal/wait epochs done, flag = "
              f"{int(bound.buffer('flags').view(torch.int32)[0])}")
        bound.close()
    ctx.close()
    comm.destroy()


if __name__ == "__main__":
    main()
