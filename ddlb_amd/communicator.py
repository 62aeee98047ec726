"""Per-process distributed runtime: device binding, RCCL process group, barrier.

Parity: ``ddlb/communicator.py:7-81`` (singleton, rank/size from env, ``set_device(local_rank)``,
``barrier() = device sync + dist.barrier()``). Differences, all MI355X/robustness driven:

* The communicator *owns* the control-plane process group (the reference's docstring claims
  so but each impl calls ``init_process_group`` itself, ``pytorch.py:53-59``). One group per
  benchmark child, RCCL (``backend="nccl"`` is RCCL on ROCm) on GPU, gloo on CPU.
* The rendezvous address comes from ``DDLB_CHILD_INIT_METHOD`` (set by the runner to a fresh
  ``tcp://addr:port`` per child, closing the port-reuse gap of SURVEY.md §5.3) or torchrun's
  ``env://`` when launched directly.
* The data plane (our own RCCL communicator, IPC symmetric memory) lives in
  :mod:`ddlb_amd.parallel` and is created lazily from this object.
* No GPU: the device falls back to CPU so the plumbing runs in CI (BASELINE config #1).
"""

from __future__ import annotations

import datetime
import os
from typing import Optional

from ddlb_amd import envs


class Communicator:
    _instance: Optional["Communicator"] = None

    def __new__(cls, *args, **kwargs):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
            cls._instance._initialized = False
        return cls._instance

    def __init__(self, device: Optional[str] = None):
        if self._initialized:
            return
        import torch

        self.rank = envs.get_rank()
        self.local_rank = envs.get_local_rank()
        self.world_size = envs.get_world_size()
        self.local_size = envs.get_local_size()
        want = device or os.environ.get("DDLB_DEVICE", "auto")
        use_gpu = (want in ("auto", "cuda", "gpu")) and torch.cuda.is_available()
        if want in ("cuda", "gpu") and not use_gpu:
            raise RuntimeError("DDLB_DEVICE=cuda requested but no ROCm GPU is visible")
        if use_gpu:
            ndev = torch.cuda.device_count()
            shared_ok = os.environ.get("DDLB_ALLOW_SHARED_GPU", "0") == "1"
            if self.local_size > ndev and not shared_ok:
                raise RuntimeError(f"local size {self.local_size} exceeds visible GPUs {ndev}")
            torch.cuda.set_device(self.local_rank % ndev)
            self.device = torch.device("cuda", self.local_rank % ndev)
            # ranks co-resident on this device (> 1 only in shared-GPU rehearsals / tests)
            self.ranks_per_device = max(1, -(-self.local_size // ndev))
        else:
            self.device = torch.device("cpu")
            self.ranks_per_device = 1
        self._native = None
        self._initialized = True

    # ------------------------------------------------------------------ properties
    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"

    @property
    def backend(self) -> str:
        """Control-plane backend: RCCL on GPU, gloo on CPU. ``DDLB_PG_BACKEND=gloo`` forces gloo
        (tests that put several ranks on one GPU, where RCCL refuses duplicate devices)."""
        forced = os.environ.get("DDLB_PG_BACKEND")
        if forced:
            return forced
        return "nccl" if self.is_gpu else "gloo"

    # ------------------------------------------------------------------ process group
    def ensure_process_group(self, timeout_s: float = 600.0):
        """Create the control-plane group once per process (idempotent)."""
        import torch.distributed as dist

        if dist.is_initialized():
            return dist.group.WORLD
        init = os.environ.get("DDLB_CHILD_INIT_METHOD")
        if init is None:
            if "MASTER_ADDR" in os.environ and "MASTER_PORT" in os.environ:
                init = "env://"
            else:
                init = f"tcp://{envs.get_master_addr()}:{envs.get_master_port()}"
        kwargs = dict(backend=self.backend, rank=self.rank, world_size=self.world_size,
                      init_method=init, timeout=datetime.timedelta(seconds=timeout_s))
        if self.is_gpu and self.backend == "nccl":
            kwargs["device_id"] = self.device
        saved = None
        if not init.startswith("env://"):
            # Under torchrun, TORCHELASTIC_USE_AGENT_STORE makes every tcp:// rendezvous assume
            # the agent hosts the store; our per-child stores are hosted by rank 0 instead.
            saved = os.environ.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        try:
            dist.init_process_group(**kwargs)
        finally:
            if saved is not None:
                os.environ["TORCHELASTIC_USE_AGENT_STORE"] = saved
        return dist.group.WORLD

    def destroy(self) -> None:
        import torch.distributed as dist

        if self._native is not None:
            try:
                self._native.close()
            except Exception:
                pass
            self._native = None
        if dist.is_available() and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass

    # ------------------------------------------------------------------ sync helpers
    def synchronize(self) -> None:
        import torch

        if self.is_gpu:
            torch.cuda.synchronize(self.device)

    def barrier(self) -> None:
        """Device sync, then a cross-rank barrier if a group exists (``communicator.py:65-74``)."""
        import torch.distributed as dist

        self.synchronize()
        if dist.is_available() and dist.is_initialized():
            if self.is_gpu and dist.get_backend() == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def host_barrier(self, tag: str = "hb") -> None:
        """A cross-rank barrier that touches no GPU queue (the process group's TCP store): for
        points where a device sync or a collective kernel would wait on work that is waiting on
        this barrier (the rccl_cap preflight's CU holders)."""
        import torch.distributed as dist

        if self.world_size <= 1 or not (dist.is_available() and dist.is_initialized()):
            return
        store = dist.distributed_c10d._get_default_store()
        self._hb_round = getattr(self, "_hb_round", 0) + 1
        key = f"ddlb_{tag}_{self._hb_round}"
        store.add(key, 1)
        import time

        t0 = time.time()
        while store.add(key, 0) < self.world_size:
            if time.time() - t0 > 120.0:
                raise TimeoutError(f"host barrier {key}: peers missing after 120 s")
            time.sleep(0.0005)

    def all_reduce_max(self, tensor):
        import torch.distributed as dist

        if self.world_size > 1 or dist.is_initialized():
            self.ensure_process_group()
            if tensor.is_cuda and dist.get_backend() != "nccl":
                host = tensor.cpu()
                dist.all_reduce(host, op=dist.ReduceOp.MAX)
                tensor.copy_(host)
            else:
                dist.all_reduce(tensor, op=dist.ReduceOp.MAX)
        return tensor

    # ------------------------------------------------------------------ data plane
    def native(self):
        """Lazily build the native data plane (own RCCL comm + IPC symmetric heap)."""
        if self._native is None:
            from ddlb_amd.parallel.context import NativeContext

            self.ensure_process_group()
            self._native = NativeContext(self)
        return self._native

    @classmethod
    def reset(cls) -> None:
        """Forget the singleton (tests / after destroy)."""
        if cls._instance is not None and cls._instance._initialized:
            cls._instance.destroy()
        cls._instance = None

    def __repr__(self) -> str:
        return (f"Communicator(rank={self.rank}, world_size={self.world_size}, "
                f"local_rank={self.local_rank}, local_size={self.local_size}, device={self.device})")
