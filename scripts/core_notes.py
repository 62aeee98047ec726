"""Post-mortem of a core file without a debugger: the signal and the instruction pointer of every
thread, symbolized.

No gdb / lldb ships in this image, so this reads the core's ELF notes directly: ``NT_PRSTATUS``
(one per thread: signal, registers) and ``NT_FILE`` (which file is mapped where), then resolves
each thread's RIP to ``library + offset`` and runs ``llvm-symbolizer`` on it. Enough to tell a
crash inside the HIP runtime from one in our own ``_C`` code. Write cores with only their notes
(``echo 0 > /proc/self/coredump_filter`` in the shell that starts the program, ``ulimit -c``
capped): a GPU process otherwise dumps gigabytes of mappings.

    python scripts/core_notes.py core.12345 [--symbolizer /opt/rocm/lib/llvm/bin/llvm-symbolizer]
"""

from __future__ import annotations

import argparse
import os
import struct
import subprocess
import sys

NT_PRSTATUS = 1
NT_FILE = 0x46494C45
PT_NOTE = 4
# x86-64 struct elf_prstatus: pr_info (3 ints) at 0, pr_cursig (short) at 12, pr_pid at 32,
# pr_reg (27 unsigned longs, user_regs_struct) at 112; rip is register 16, rsp 19
_PR_REG = 112
_REGS = ("r15 r14 r13 r12 rbp rbx r11 r10 r9 r8 rax rcx rdx rsi rdi orig_rax rip cs eflags rsp "
         "ss fs_base gs_base ds es fs gs").split()


def notes(data: bytes):
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise SystemExit("not a 64-bit ELF core")
    phoff, = struct.unpack_from("<Q", data, 0x20)
    phentsize, phnum = struct.unpack_from("<HH", data, 0x36)
    for i in range(phnum):
        ptype, _, off, _, _, filesz = struct.unpack_from("<IIQQQQ", data, phoff + i * phentsize)
        if ptype != PT_NOTE:
            continue
        pos, end = off, min(off + filesz, len(data))
        while pos + 12 <= end:
            namesz, descsz, ntype = struct.unpack_from("<III", data, pos)
            pos += 12
            pos += (namesz + 3) & ~3
            desc = data[pos:pos + descsz]
            pos += (descsz + 3) & ~3
            yield ntype, desc


def parse_files(desc: bytes):
    count, page = struct.unpack_from("<QQ", desc, 0)
    ents = [struct.unpack_from("<QQQ", desc, 16 + 24 * i) for i in range(count)]
    names = desc[16 + 24 * count:].split(b"\0")
    return [(s, e, off * page, names[i].decode(errors="replace")) for i, (s, e, off) in
            enumerate(ents)]


def resolve(addr: int, files):
    for s, e, off, name in files:
        if s <= addr < e:
            return name, addr - s + off
    return None, None


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("core")
    ap.add_argument("--symbolizer", default="/opt/rocm/lib/llvm/bin/llvm-symbolizer")
    a = ap.parse_args()
    with open(a.core, "rb") as f:
        data = f.read()
    threads, files = [], []
    for ntype, desc in notes(data):
        if ntype == NT_PRSTATUS and len(desc) >= _PR_REG + 8 * len(_REGS):
            signo, = struct.unpack_from("<i", desc, 0)
            cursig, = struct.unpack_from("<h", desc, 12)
            pid, = struct.unpack_from("<i", desc, 32)
            regs = dict(zip(_REGS, struct.unpack_from("<" + "Q" * len(_REGS), desc, _PR_REG)))
            threads.append((pid, cursig or signo, regs))
        elif ntype == NT_FILE:
            files = parse_files(desc)
    print(f"{a.core}: {len(threads)} threads, {len(files)} file mappings")
    for pid, sig, regs in threads:
        rip = regs["rip"]
        name, off = resolve(rip, files)
        where = f"{os.path.basename(name)}+{off:#x}" if name else "?"
        sym = ""
        if name and os.path.exists(a.symbolizer) and os.path.exists(name):
            try:
                out = subprocess.run([a.symbolizer, "--obj", name, "--demangle", hex(off)],
                                     capture_output=True, text=True, timeout=60).stdout
                sym = " | ".join(x for x in out.splitlines() if x.strip())[:300]
            except (OSError, subprocess.SubprocessError):
                pass
        flag = "  <== signal" if sig else ""
        print(f"tid {pid} sig {sig} rip {rip:#x} {where} {sym}{flag}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
