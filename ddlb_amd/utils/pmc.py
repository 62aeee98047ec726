"""Opt-in PMC (hardware counter) collection for the benchmark runner.

The reference's only profiling hook is the 5-iteration ``cudaProfilerStart/Stop`` window that an
external ``nsys --capture-range=cudaProfilerApi`` records (``ddlb/benchmark.py:89-104``). Here the
same window is delimited with ``roctxProfilerResume/Pause`` (``ddlb_amd.utils.profiling``), and
``--pmc SQ_WAVES,...`` makes the runner start each benchmark child under
``rocprofv3 --pmc <counters> --selected-regions`` and the per-kernel means come back in the CSV row
(``pmc`` column, JSON; the 8 kernels with the most GPU-active cycles). Measured on this image
(``profiles/r03/r3_8_cli_pmc_default_set.txt``): rocprofv3 counted every dispatch of the child, not
only the window's five ``run()`` calls, so a row's means also include the warmup / timed runs of
the same kernels (and its validation kernels, which the per-kernel split keeps apart).

rocprofv3 does not split counters over passes, and asking one pass for more than the hardware
blocks hold makes it hang (``error code 38``) — so the set is checked against the per-pass limits
of MI355X before anything is launched (``MI355X_MICROARCH.md`` §Profiling: 8 SQ, 4 TCC (FETCH_SIZE
takes 3, WRITE_SIZE 2), 4 TCP, 2 TA, 2 TD, 2 GRBM; ``_sum``/``_avr``/``_min``/``_max`` of one
counter count once).
"""

from __future__ import annotations

import collections
import os
import re
import shutil
import sqlite3
from typing import Dict, List, Sequence

BLOCK_LIMITS = {"SQ": 8, "TCC": 4, "TCP": 4, "TA": 2, "TD": 2, "GRBM": 2}
#: derived counters that occupy several hardware slots of one block
DERIVED_SLOTS = {"FETCH_SIZE": ("TCC", 3), "WRITE_SIZE": ("TCC", 2)}
#: a useful default pass: MFMA work and busy cycles, LDS pressure, waits
DEFAULT_SET = ("SQ_WAVES", "SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_VALU_MFMA_BUSY_CYCLES",
               "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES",
               "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")


def parse(spec) -> List[str]:
    """``"a,b c"`` or a sequence -> counter names (``"default"`` = :data:`DEFAULT_SET`)."""
    if spec in (None, "", False):
        return []
    if isinstance(spec, str):
        if spec.strip() == "default":
            return list(DEFAULT_SET)
        return [c for c in re.split(r"[,\s]+", spec) if c]
    return [str(c) for c in spec]


def _base(name: str) -> str:
    return re.sub(r"_(sum|avr|min|max)$", "", name)


def check_limits(counters: Sequence[str]) -> Dict[str, int]:
    """Slots used per hardware block; raises ValueError when one pass cannot hold the set."""
    used: Dict[str, int] = collections.Counter()
    seen = set()
    for c in counters:
        b = _base(c)
        if b in seen:
            continue
        seen.add(b)
        if b in DERIVED_SLOTS:
            blk, n = DERIVED_SLOTS[b]
            used[blk] += n
            continue
        blk = b.split("_", 1)[0]
        if blk not in BLOCK_LIMITS:
            raise ValueError(f"counter {c}: unknown block {blk} (known: {sorted(BLOCK_LIMITS)})")
        used[blk] += 1
    over = {b: n for b, n in used.items() if n > BLOCK_LIMITS[b]}
    if over:
        raise ValueError("one rocprofv3 pass cannot hold these counters ("
                         + ", ".join(f"{b}: {n} > {BLOCK_LIMITS[b]}" for b, n in over.items())
                         + "); split them over several runs")
    return dict(used)


def rocprof_cmd(counters: Sequence[str], out_dir: str, name: str = "pmc") -> List[str]:
    """Launcher prefix: the program itself must follow ``--`` (no env / shell hop: the
    profiler's preloaded library has initialised the GPU by then)."""
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    return [exe, "--pmc", *counters, "--selected-regions", "-d", out_dir, "-o", name, "--"]


def summarize(out_dir: str, match: str = "", top: int = 0) -> Dict[str, Dict[str, float]]:
    """Per kernel (short name): mean of every counter over the recorded dispatches; ``top`` > 0
    keeps the kernels with the most ``GRBM_GUI_ACTIVE`` (else ``SQ_WAVE_CYCLES``) only."""
    vals: Dict[str, Dict[str, List[float]]] = collections.defaultdict(
        lambda: collections.defaultdict(list))
    for root, _, files in os.walk(out_dir):
        for f in files:
            if not f.endswith(".db"):
                continue
            con = sqlite3.connect(os.path.join(root, f))
            try:
                tables = {r[0] for r in con.execute("select name from sqlite_master")}
                if "counters_collection" not in tables:
                    continue
                for kn, cn, v in con.execute(
                        "select kernel_name, counter_name, value from counters_collection"):
                    if match in kn:
                        vals[short_name(kn)][cn].append(float(v))
            finally:
                con.close()
    out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
    if top > 0 and len(out) > top:
        def weight(item):
            cs = item[1]
            return cs.get("GRBM_GUI_ACTIVE", cs.get("SQ_WAVE_CYCLES", 0.0))
        out = dict(sorted(out.items(), key=weight, reverse=True)[:top])
    return out


def short_name(name: str) -> str:
    if name.startswith("Custom_Cijk") or name.startswith("Cijk"):
        return "hipBLASLt " + name.split("_MT")[1].split("_")[0] if "_MT" in name else name[:60]
    base = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    return re.sub(r"^.*::", "", base.split("<")[0]) + ("<" + base.split("<", 1)[1]
                                                       if "<" in base else "")
