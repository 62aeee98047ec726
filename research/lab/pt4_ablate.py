"""pt4 ablation lab: build text-patched copies of the product GEMM header and time them against
the unpatched kernel, interleaved in ONE process (cdna guide §5.4 rule 24).

The product kernel stays free of ablation switches: every variant here is the product header
(``csrc/gemm/gemm_kernels.h``) with a few textual substitutions, compiled into its own shared
object (``research/lab/pt4_lab.hip`` is the entry point). Build on the CPU host (hipcc
cross-compiles gfx950), then time on the GPU box::

    python research/lab/pt4_ablate.py --build-only                 # here
    python research/lab/pt4_ablate.py --variants base,nostore      # on the GPU

Variants (TIMING-ONLY unless marked exact):
  base      the product kernel, unchanged (exact; checked against the fp32 product)
  ref       the product kernel as committed at git revision $DDLB_LAB_REF (default HEAD): the
            A/B partner of an edited kernel (exact; checked)
  nostore   no C stores at all: the store instructions are replaced by a keep-alive of their
            operands and the vmcnt windows that counted them shrink to the DMA alone
  l2store   C stores with the default (write-back) policy into one 128 KB region per XCD group
            (blocks b and b + 8 share it): the same store instructions, no HBM write stream
            (the parked quarter still goes to C as in the product)
  dmam      the B unit's LDS-DMA issued at the head of the MFMA phase instead of in the load
            phase (exact); dmam1 the same at MFMA priority
  lgkm_g0   wave group 0 waits for its fragment reads after the barrier, not before (exact)
  auxN      the product kernel with C store cache-policy bits N (exact)
  behind    store-behind (exact; research/lab/pt4_store_behind.diff, round 6, measured slower:
            profiles/r06/README.md): a tile's C packed into held registers and stored over three
            intervals of the next tile instead of one
  ring      A in a 3-deep ring of K-tile slots (exact; research/lab/pt4_a_ring.diff, round 6,
            160 KB LDS, A staged three K-tiles ahead): within 1 % everywhere, slower on square
            shapes (profiles/r06/README.md, r6_6)
  hold      8 of 16 C stores per wave beside the next tile's MFMAs: 4 held in registers (K-tile
            0), 4 parked (K-tile 1, under a run-time flag) (exact; research/lab/pt4_hold.diff,
            round 6: slower, r6_11)
  nodma / noread / nomfma  the iterations without their operand DMA / fragment reads / MFMAs
            (TIMING-ONLY): what each costs the steady K-tile
  hold0     the 4 held pairs and the 4 parked ones all stored in the next tile's K-tile 0 (exact;
            research/lab/pt4_hold0.diff, round 6: 1.3-1.4 % slower, r6_16)
  relax     the first K-tile after a tile's C stores waits for them only as far as the DMA it
            needs requires (exact)
  stagG_Dk  workgroup slot (blockIdx / 8) mod G starts slot x D thousand shader cycles late
            (exact): do desynchronized tile ends (C write bursts of fewer CUs at a time) pay for
            the delay?
  dmafirst  each load phase issues its 4 LDS-DMA pieces before its 12 fragment reads (exact);
            dmamid between the B and the A reads
  noprio    the MFMA phases without s_setprio 1 (exact)
  lgkm0     lgkm_g0 on the park kernel: wave group 0's fragment-read wait left to the compiler's
            waits at the consuming MFMAs, after the barrier (exact)
  prioload  the load phases at wave priority 2 (exact)
  al2       TIMING-ONLY: every tile reads its A from one of two 256-row panels (L2-resident at
            K = 1024), C unchanged; al2ns the same without C stores
  krot      workgroup slot (blockIdx / 8) mod 4 starts each tile's K loop a quarter further in
            (exact up to summation order): the CUs sharing an A panel stop fetching it in lockstep
  mrot      tile (tm, tn) starts its K loop at K-tile tm mod nk (exact up to summation order):
            the A-panel sharers stay in lockstep, concurrent M-blocks fetch different K offsets
  nocross   the steady K-loop without the tile-crossing test in stage() (exact): all of a tile's
            loop iterations but the last stage K-tiles of that tile
  g1split   the body instantiated once per wave group (exact): the per-phase `if (g1)` branches
            around the vmcnt waits fold away
  m0share   the second 1 KB piece of each unit slice addressed through the DMA's instruction
            offset (exact iff that offset also applies to the LDS address): half the M0 writes
  waitall   steady K-tiles wait on vmcnt in both wave groups at all four sites (exact): no
            per-phase branch, no second copy of the loop
  unroll2   the steady loop unrolled by two (exact)
  pstamps   the product kernel without the C park (exact), tagged s_memtime stamps by waves 0
            and 4 after each barrier (0), after a load phase's DMA issue (1), after an MFMA
            phase's last MFMA issue (2) and before each barrier (3): which side of a barrier waits
            (--stamp-report prints the per-phase breakdown)
  stamps    the product kernel without the C park (exact) with an s_memtime stamp after every workgroup barrier by
            waves 0 and 4, kept in 8 KB of LDS beside the staging buffers (no vmcnt traffic) and
            written to the debug buffer at the end: [block][group][512] u64, entry 0 / 1 =
            s_memrealtime at start / end, 2 = stamp count, 3.. = stamps
"""

from __future__ import annotations

import argparse
import ctypes
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "csrc", "gemm")
BIN = os.path.join(HERE, "bin")
WORK = os.path.join(ROOT, "build", "lab")

_STORE_PAIR = ("""          __builtin_amdgcn_raw_buffer_store_b128(x, crc, c_pair, so, CPOL);
          __builtin_amdgcn_raw_buffer_store_b128(y, crc, c_pair, so8, CPOL);""")
_SO = """          const unsigned so = (unsigned)((prow * p.ldc + cn0) * OSZ) + (KS ? ccs : 0u);"""

_STAMP_DEF = """  const bool g1 = wr == 1;  // wave-uniform (wave came through readfirstlane)
  // lab: stamps after every barrier, waves 0 and 4, in LDS past the staging buffers
  int lab_i = 3;
  const uint64_t lab_t0 = __builtin_amdgcn_s_memrealtime();
  auto lab_stamp = [&]() __attribute__((always_inline)) {
    if ((wave & 3) == 0 && lab_i < 512) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      *(uint64_t*)(smem + 8 * UNIT + (wave >> 2) * 4096 + lab_i * 8) = t;
    }
    ++lab_i;
  };
#undef T4_BAR
#define T4_BAR()                         \\
  do {                                   \\
    __builtin_amdgcn_sched_barrier(0);   \\
    __builtin_amdgcn_s_barrier();        \\
    __builtin_amdgcn_sched_barrier(0);   \\
    lab_stamp();                         \\
    __builtin_amdgcn_sched_barrier(0);   \\
  } while (0)"""
_STAMP_END = """  wait_vm<0>();  // never leave an LDS-DMA in flight past the end of the workgroup
  if ((wave & 3) == 0) {  // lab: stamps out
    uint64_t* d = (uint64_t*)p.timeout_word + ((int64_t)blockIdx.x * 2 + (wave >> 2)) * 512;
    const uint64_t* src = (const uint64_t*)(smem + 8 * UNIT + (wave >> 2) * 4096);
    for (int e = 3 + lane; e < (lab_i < 512 ? lab_i : 512); e += 64) d[e] = src[e];
    if (lane == 0) {
      d[0] = lab_t0;
      d[1] = __builtin_amdgcn_s_memrealtime();
      d[2] = (uint64_t)lab_i;
    }
  }"""

_PSTAMP_DEF = """  const bool g1 = wr == 1;  // wave-uniform (wave came through readfirstlane)
  // lab: tagged stamps (t << 4 | tag) by waves 0 and 4 in LDS past the staging buffers:
  // 0 after a barrier, 1 after a load phase's DMA issue, 2 after an MFMA phase's last MFMA
  // issue, 3 before a barrier (the phase's waits done)
  int lab_i = 3;
  const uint64_t lab_t0 = __builtin_amdgcn_s_memrealtime();
  auto lab_stamp = [&](int tag) __attribute__((always_inline)) {
    if ((wave & 3) == 0 && lab_i < 512) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      *(uint64_t*)(smem + 8 * UNIT + (wave >> 2) * 4096 + lab_i * 8) = (t << 4) | (uint64_t)tag;
    }
    ++lab_i;
  };
#undef T4_BAR
#define T4_BAR()                         \\
  do {                                   \\
    __builtin_amdgcn_sched_barrier(0);   \\
    lab_stamp(3);                        \\
    __builtin_amdgcn_sched_barrier(0);   \\
    __builtin_amdgcn_s_barrier();        \\
    __builtin_amdgcn_sched_barrier(0);   \\
    lab_stamp(0);                        \\
    __builtin_amdgcn_sched_barrier(0);   \\
  } while (0)"""
_SB = "__builtin_amdgcn_sched_barrier(0);"

PATCHES = {
    "base": [],
    "ref": [],
    "behind": [],
    "ring": [],
    "hold": [],
    "hold0": [],
    "nostore": [
        ("constexpr int NS = 4 * Store8<OUT>::kStores;", "constexpr int NS = 0;"),
        ("  constexpr int NP = PARK ? 4 : 0;", "  constexpr int NP = 0;  // lab"),
        (_STORE_PAIR, """          asm volatile("" ::"v"(x), "v"(y), "s"(so), "s"(so8));"""),
        ("      __builtin_amdgcn_raw_buffer_store_b128(v[jj], crc, c_pair, so, CPOL);",
         '      asm volatile("" ::"v"(v[jj]), "s"(so));  // lab'),
    ],
    "l2store": [
        (_SO, """          const unsigned so = (unsigned)((((int64_t)(blockIdx.x % 8) * 256 + mq * 64 + f * 16) *
                                           p.ldc) * OSZ);  // lab: one region per XCD group"""),
        (_STORE_PAIR, """          __builtin_amdgcn_raw_buffer_store_b128(x, crc, c_pair, so, 0);  // lab: write-back
          __builtin_amdgcn_raw_buffer_store_b128(y, crc, c_pair, so8, 0);"""),
    ],
    # the B unit's LDS-DMA (2 of the 4 ops a wave issues per load phase) moved from the load
    # phase to the head of the wave's next MFMA phase (g1's waits after its load phases drop by
    # the 2 ops issued after them; g0's waits after its MFMA phases keep their counts)
    **{name: [
        ("""      stage(0, 1, BUF ^ 1, qa);
      stage(1, 1, BUF ^ 1, qa);
      T4_LGKM0();
      if (g1) wait_vm<KIND == 2 ? 8 + 3 * NS : 8>();
      T4_BAR();
      __builtin_amdgcn_s_setprio(1);
      if constexpr (DEF) mm(1, 1, false);""", """      stage(0, 1, BUF ^ 1, qa);
      T4_LGKM0();
      if (g1) wait_vm<KIND == 2 ? 6 + 3 * NS : 6>();
      T4_BAR();
""" + ("      __builtin_amdgcn_s_setprio(1);\n" if prio else "") + """      stage(1, 1, BUF ^ 1, qa);  // lab
      __builtin_amdgcn_s_setprio(1);
      if constexpr (DEF) mm(1, 1, false);"""),
        ("""      stage(0, 0, BUF, qb);
      stage(1, 0, BUF, qb);
      T4_LGKM0();
      if (g1) wait_vm<KIND == 1 && !PAIRST ? 8 + NS : 8>();
      T4_BAR();
      __builtin_amdgcn_s_setprio(1);
      mm(0, 1, Z);""", """      stage(0, 0, BUF, qb);
      T4_LGKM0();
      if (g1) wait_vm<KIND == 1 && !PAIRST ? 6 + NS : 6>();
      T4_BAR();
""" + ("      __builtin_amdgcn_s_setprio(1);\n" if prio else "") + """      stage(1, 0, BUF, qb);  // lab
      __builtin_amdgcn_s_setprio(1);
      mm(0, 1, Z);"""),
    ] for name, prio in (("dmam", False), ("dmam1", True))},
    # wave group 0 retires its fragment reads after the barrier instead of before it (its reads'
    # WAR partner, g1's DMA into the same unit, comes 3 intervals later; g1's reads keep the
    # lgkmcnt before the barrier: g0 restages their unit 1 interval later)
    "lgkm_g0": [
        ("""      T4_LGKM0();
      if (g1) wait_vm<KIND == 2 ? 8 + 3 * NS : 8>();
      T4_BAR();""", """      if (g1) {  // lab
        T4_LGKM0();
        wait_vm<KIND == 2 ? 8 + 3 * NS : 8>();
        T4_BAR();
      } else {
        T4_BAR();
        T4_LGKM0();
      }"""),
        ("""      T4_LGKM0();
      if (g1) wait_vm<KIND == 1 && !PAIRST ? 8 + NS : 8>();
      T4_BAR();""", """      if (g1) {  // lab
        T4_LGKM0();
        wait_vm<KIND == 1 && !PAIRST ? 8 + NS : 8>();
        T4_BAR();
      } else {
        T4_BAR();
        T4_LGKM0();
      }"""),
    ],
    # C store cache policy (aux bits of buffer_store: 1 sc0, 2 nt, 16 sc1; the product uses 18,
    # 17 for MX-fp8)
    **{f"aux{a}": [(_STORE_PAIR, f"""          __builtin_amdgcn_raw_buffer_store_b128(x, crc, c_pair, so, {a});  // lab
          __builtin_amdgcn_raw_buffer_store_b128(y, crc, c_pair, so8, {a});""")]
       for a in (0, 1, 3, 17, 18, 19)},
    # where the steady K-tile's time goes (TIMING-ONLY, wrong results): no operand DMA in the
    # iterations (the prologue's stays), no fragment reads, no MFMAs (operands kept alive)
    "nodma": [
        ("      stage_ab(same_tag, 1, BUF ^ 1, qa);\n      T4_LGKM0();\n"
         "      if constexpr (PARK", "      T4_LGKM0();\n      if constexpr (PARK"),
        ("      stage_ab(same_tag, 0, BUF, qb);\n      T4_LGKM0();\n"
         "      if constexpr (PARK", "      T4_LGKM0();\n      if constexpr (PARK"),
    ],
    "noread": [
        ("      loadB(bufc, 0);  // phase A: halves 0\n      loadA(bufc, 0);\n      if constexpr (PARK",
         "      if constexpr (PARK"),
        ("      loadB(bufc, 1);  // phase B: halves 1\n      loadA(bufc, 1);\n      if constexpr (PARK",
         "      if constexpr (PARK"),
    ],
    "nomfma": [
        ("          Mma::step8(acc[mq * 4 + f][nq * 2 + g], bP[nq][g], aP[h][f]);",
         '          asm volatile("" ::"v"(bP[nq][g]), "v"(aP[h][f]));  // lab'),
        ("            Mma::step(acc[mq * 4 + f][nq * 2 + g], bR[nq][g][kk], aR[h][f][kk]);",
         '            asm volatile("" ::"v"(bR[nq][g][kk]), "v"(aR[h][f][kk]));  // lab'),
    ],
    # MFMAs and barriers only
    "mfmaonly": "nodma+noread",
    # the first K-tile of a tile (KIND 2) keeps the previous tile's C stores in flight up to the
    # exact counts (PAIRST: 8 + 4 NS at all four waits) instead of 8 + 3 NS / 8
    "relax": [
        ("if (g1) wait_vm<KIND == 2 ? 8 + 3 * NS : 8>();",
         "if (g1) wait_vm<KIND == 2 ? (PAIRST ? 8 + 4 * NS : 8 + 3 * NS) : 8>();  // lab"),
        ("if (!g1) wait_vm<KIND == 2 ? 8 + 3 * NS : (KIND == 1 && !PAIRST ? 8 + NS : 8)>();",
         "if (!g1) wait_vm<KIND == 2 ? (PAIRST ? 8 + 4 * NS : 8 + 3 * NS) : "
         "(KIND == 1 && !PAIRST ? 8 + NS : 8)>();  // lab"),
        ("if (g1) wait_vm<KIND == 1 && !PAIRST ? 8 + NS : 8>();",
         "if (g1) wait_vm<KIND == 2 && PAIRST ? 8 + 4 * NS : (KIND == 1 && !PAIRST ? 8 + NS : 8)>();"),
        ("if (!g1) wait_vm<KIND == 1 ? 8 + 4 * NS : 8>();",
         "if (!g1) wait_vm<KIND == 1 || (KIND == 2 && PAIRST) ? 8 + 4 * NS : 8>();  // lab"),
    ],
    # desynchronized tile phases (TIMING-ONLY probe, exact results): workgroup slot g = (bid / 8)
    # mod G (every XCD holds every slot) starts g * D shader cycles late, so the CUs' C write
    # bursts stop coinciding; the delay is paid at the end
    **{f"stag{g}_{d // 1000}k": [
        ("  if (my_tiles == 0) return;\n", f"""  if (my_tiles == 0) return;
  {{  // lab: stagger
    const uint64_t lab_d = (uint64_t)((bid >> 3) % {g}) * {d}u;
    const uint64_t lab_t = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - lab_t < lab_d) __builtin_amdgcn_s_sleep(2);
  }}
""")] for g, d in ((2, 3000), (2, 6000), (2, 12000), (4, 3000))},
    # load-phase order (exact): the 4 LDS-DMA pieces issued before the 12 fragment reads
    # (dmafirst) or between the B and the A reads (dmamid). The DMA writes units no read of the
    # phase touches, and the vmcnt counts stay (the DMA still precedes the parked stores)
    **{name: [
        ("""      loadB(bufc, 0);  // phase A: halves 0
      loadA(bufc, 0);
      if constexpr (PARK && KIND == 2) park_read(0, pv);
      stage(0, 1, BUF ^ 1, qa);
      stage(1, 1, BUF ^ 1, qa);
""", pre + """      stage(0, 1, BUF ^ 1, qa);  // lab
      stage(1, 1, BUF ^ 1, qa);
""" + post.replace("@", "0") + """      if constexpr (PARK && KIND == 2) park_read(0, pv);
"""),
        ("""      loadB(bufc, 1);  // phase B: halves 1
      loadA(bufc, 1);
      if constexpr (PARK && KIND == 2) park_read(2, pv);
      stage(0, 0, BUF, qb);
      stage(1, 0, BUF, qb);
""", pre.replace("0);", "1);") + """      stage(0, 0, BUF, qb);  // lab
      stage(1, 0, BUF, qb);
""" + post.replace("@", "1") + """      if constexpr (PARK && KIND == 2) park_read(2, pv);
"""),
    ] for name, pre, post in (
        ("dmafirst", "", "      loadB(bufc, @);\n      loadA(bufc, @);\n"),
        ("dmamid", "      loadB(bufc, 0);\n", "      loadA(bufc, @);\n"))},
    # no wave priority: the MFMA phases without s_setprio 1 (exact)
    "noprio": [
        ("      __builtin_amdgcn_s_setprio(1);\n      if constexpr (DEF) mm(1, 1, false);",
         "      if constexpr (DEF) mm(1, 1, false);  // lab"),
        ("      __builtin_amdgcn_s_setprio(1);\n      mm(0, 1, Z);", "      mm(0, 1, Z);  // lab"),
    ],
    # lgkm_g0 on the park kernel (exact): wave group 0 leaves its fragment-read wait to the
    # compiler's waits at the MFMAs that consume them, after the barrier
    "lgkm0": [
        ("""      T4_LGKM0();
      if constexpr (PARK && KIND == 2) park_store(0, pv);""",
         """      if (g1) T4_LGKM0();  // lab
      if constexpr (PARK && KIND == 2) park_store(0, pv);"""),
        ("""      T4_LGKM0();
      if constexpr (PARK && KIND == 2) park_store(2, pv);""",
         """      if (g1) T4_LGKM0();  // lab
      if constexpr (PARK && KIND == 2) park_store(2, pv);"""),
    ],
    # load phases at wave priority 2, above either MFMA phase (exact)
    "prioload": [
        ("      loadB(bufc, 0);  // phase A: halves 0\n",
         "      __builtin_amdgcn_s_setprio(2);  // lab\n      loadB(bufc, 0);\n"),
        ("      if (g1) wait_vm<KIND == 2 ? WK2A : 8>();\n      T4_BAR();\n",
         "      if (g1) wait_vm<KIND == 2 ? WK2A : 8>();\n"
         "      __builtin_amdgcn_s_setprio(0);  // lab\n      T4_BAR();\n"),
        ("      loadB(bufc, 1);  // phase B: halves 1\n",
         "      __builtin_amdgcn_s_setprio(2);  // lab\n      loadB(bufc, 1);\n"),
        ("      if (g1) wait_vm<KIND == 2 ? WK2B : (KIND == 1 && !PAIRST ? 8 + NS : 8)>();\n"
         "      T4_BAR();\n",
         "      if (g1) wait_vm<KIND == 2 ? WK2B : (KIND == 1 && !PAIRST ? 8 + NS : 8)>();\n"
         "      __builtin_amdgcn_s_setprio(0);  // lab\n      T4_BAR();\n"),
    ],
    # TIMING-ONLY: every tile's A operand read from one of two 256-row panels (L2-resident at
    # K = 1024 beside the 2 MB B), the C stores unchanged: what the A stream from HBM costs
    "al2": [
        ("rsA = __builtin_amdgcn_make_buffer_rsrc((void*)((APAN ? na : a_panel(nm0)) + (KS ? nko : 0)),",
         "rsA = __builtin_amdgcn_make_buffer_rsrc((void*)((APAN ? na : a_panel(((nm0 >> 8) & 1) * 256)) + (KS ? nko : 0)),  // lab"),
    ],
    "al2ns": "al2+nostore",
    # K-rotation (exact up to f32 summation order): workgroup slot (blockIdx / 8) mod 4 -- the
    # four CUs that share an A panel on the flagship -- starts every tile's K loop a quarter of
    # the way in, so one of them fetches each A K-tile from HBM and the others find it in L2
    "krot": [
        ("    const unsigned soff = (unsigned)(c.kt * ROWB);",
         """    int lab_k = c.kt + (((int)blockIdx.x >> 3) & 3) * (nk >> 2);  // lab
    if (lab_k >= nk) lab_k -= nk;
    const unsigned soff = (unsigned)(lab_k * ROWB);"""),
    ],
    # K-rotation by M-block (exact up to summation order): tile (tm, tn) starts its K loop at
    # K-tile tm mod nk, so the four CUs sharing an A panel stay in lockstep while concurrent
    # M-blocks fetch different K offsets (rows lda apart: a power-of-two stride puts every
    # concurrent A line of the chip at the same low address bits)
    "mrot": [
        ("  int src_tile = -1;\n", "  int src_tile = -1;\n  int lab_nrot = 0, lab_srot = 0;  // lab\n"),
        ("    if constexpr (APAN) na = a_panel(m0);\n",
         "    if constexpr (APAN) na = a_panel(m0);\n    lab_nrot = (int)((m0 >> 8) % nk);  // lab\n"),
        ("      src_tile = c.ti;\n", "      src_tile = c.ti;\n      lab_srot = lab_nrot;  // lab\n"),
        ("    const unsigned soff = (unsigned)(c.kt * ROWB);",
         """    int lab_k = c.kt + lab_srot;  // lab
    if (lab_k >= nk) lab_k -= nk;
    const unsigned soff = (unsigned)(lab_k * ROWB);"""),
    ],
    # the steady K-loop without the tile-crossing check (exact): every iteration but the last of
    # a tile's loop stages K-tiles of the same tile, so its stage() skips the descriptor rebuild
    # test (8 s_cselect per load phase) and its cursor advance is ++kt
    "nocross": [
        ("  };\n  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;\n",
         """  };
  auto stage_nc = [&](int X, int q, int buf, Cur c) __attribute__((always_inline)) {  // lab
    const unsigned* off = X == 0 ? offA[q] : offB[q];
    char* dst = smem + uoff(X, buf, q) + wave * 16 * ROWB;
    const unsigned soff = (unsigned)(c.kt * ROWB);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)dst, 16, off[0],
                                             soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)(dst + 8 * ROWB),
                                             16, off[1], soff, 0, 0);
  };
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
"""),
        ("  auto iter = [&](auto bufc, auto kind_tag) __attribute__((always_inline)) {\n",
         "  auto iter = [&](auto bufc, auto kind_tag, auto nc_tag) __attribute__((always_inline)) {\n"
         "    constexpr bool NC = decltype(nc_tag)::value;  // lab\n"),
        ("      stage(0, 1, BUF ^ 1, qa);\n      stage(1, 1, BUF ^ 1, qa);\n      T4_LGKM0();\n"
         "      if constexpr (PARK && KIND == 2) park_store(0, pv);",
         """      if constexpr (NC) {  // lab
        stage_nc(0, 1, BUF ^ 1, qa);
        stage_nc(1, 1, BUF ^ 1, qa);
      } else {
        stage(0, 1, BUF ^ 1, qa);
        stage(1, 1, BUF ^ 1, qa);
      }
      T4_LGKM0();
      if constexpr (PARK && KIND == 2) park_store(0, pv);"""),
        ("      stage(0, 0, BUF, qb);\n      stage(1, 0, BUF, qb);\n      T4_LGKM0();\n"
         "      if constexpr (PARK && KIND == 2) park_store(2, pv);",
         """      if constexpr (NC) {  // lab
        stage_nc(0, 0, BUF, qb);
        stage_nc(1, 0, BUF, qb);
      } else {
        stage(0, 0, BUF, qb);
        stage(1, 0, BUF, qb);
      }
      T4_LGKM0();
      if constexpr (PARK && KIND == 2) park_store(2, pv);"""),
        ("    qa = qb;\n    adv(qb);\n  };\n",
         "    qa = qb;\n    if constexpr (NC) ++qb.kt; else adv(qb);  // lab\n  };\n"),
        ("""    iter(B0{}, first_kind);  // K-tile 0
    for (int t = 1; t + 2 < nk; t += 2) {
      iter(B1{}, K0{});
      iter(B0{}, K0{});
    }
    iter(B1{}, last_kind);  // K-tile nk - 1 (nk even)""",
         """    using NCT = std::true_type;  // lab
    using NCF = std::false_type;
    iter(B0{}, first_kind, NCF{});  // K-tile 0
    int t = 1;
    for (; t + 4 < nk; t += 2) {  // qb <= K-tile t + 3 <= nk - 2: the same tile
      iter(B1{}, K0{}, NCT{});
      iter(B0{}, K0{}, NCT{});
    }
    if (t + 2 < nk) {
      iter(B1{}, K0{}, NCF{});
      iter(B0{}, K0{}, NCF{});
    }
    iter(B1{}, last_kind, NCF{});  // K-tile nk - 1 (nk even)"""),
    ],
    # the wave groups' code split at compile time (exact): the body after the prologue's
    # setup is instantiated once per wave group, so `if (g1)` around the vmcnt waits folds away
    # (no branch per phase)
    "g1split": [
        ("  const bool g1 = wr == 1;  // wave-uniform (wave came through readfirstlane)\n",
         "  auto lab_body = [&](auto g1_tag) __attribute__((always_inline)) {  // lab\n"
         "  constexpr bool g1 = decltype(g1_tag)::value;\n"),
        ("#undef T4_BAR\n#undef T4_LGKM0\n  wait_vm<0>();",
         "  };  // lab\n  if (wr == 1)\n    lab_body(std::true_type{});\n  else\n"
         "    lab_body(std::false_type{});\n#undef T4_BAR\n#undef T4_LGKM0\n  wait_vm<0>();"),
    ],
    # one M0 per unit (exact if the DMA's instruction offset also offsets its LDS address): the
    # second 1 KB piece of a wave's unit slice takes the first's LDS base with offset:1024 and a
    # voffset 1024 lower, so the compiler needs 2 M0 writes (and s_nops) per load phase, not 4
    "m0share": [
        ("      offB[q][i] = (unsigned)(lc * p.ldb * esz + ch);\n",
         "      offB[q][i] = (unsigned)(lc * p.ldb * esz + ch);\n"
         "      if (i == 1) {  // lab: rows 8.. of the slice are >= 8 rows in, so >= 1024 bytes\n"
         "        offA[q][i] -= 1024u;\n        offB[q][i] -= 1024u;\n      }\n"),
        ("""    __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)(dst + 8 * ROWB),
                                             16, off[1], soff, 0, 0);""",
         """    __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)dst,  // lab
                                             16, off[1], soff, 8 * ROWB, 0);"""),
    ],
    # branch-free steady K-tiles (exact): in KIND 0 iterations both wave groups wait at all four
    # vmcnt sites (same count 8: group 1 gains no-op waits, group 0 waits for its DMA one interval
    # earlier), so the per-phase `if (g1)` branch disappears without a second copy of the loop
    "waitall": [
        ("      if (g1) wait_vm<KIND == 2 ? WK2A : 8>();",
         "      if (KIND == 0 || g1) wait_vm<KIND == 2 ? WK2A : 8>();  // lab"),
        ("      if (!g1) wait_vm<KIND == 2 ? WK2A : (KIND == 1 && !PAIRST ? 8 + NS : 8)>();",
         "      if (KIND == 0 || !g1) wait_vm<KIND == 2 ? WK2A : (KIND == 1 && !PAIRST ? 8 + NS : 8)>();  // lab"),
        ("      if (g1) wait_vm<KIND == 2 ? WK2B : (KIND == 1 && !PAIRST ? 8 + NS : 8)>();",
         "      if (KIND == 0 || g1) wait_vm<KIND == 2 ? WK2B : (KIND == 1 && !PAIRST ? 8 + NS : 8)>();  // lab"),
        ("      if (!g1) wait_vm<KIND == 1 ? 8 + 4 * NS - NP : (KIND == 2 ? WK2B : 8)>();",
         "      if (KIND == 0 || !g1) wait_vm<KIND == 1 ? 8 + 4 * NS - NP : (KIND == 2 ? WK2B : 8)>();  // lab"),
    ],
    # the steady loop unrolled by two (4 K-tiles per trip: half the loop-control instructions
    # and back branches) (exact)
    "unroll2": [
        ("    for (; t + 4 < nk; t += 2) {  // qb <= K-tile t + 3 <= nk - 2: this tile\n",
         "#pragma unroll 2\n    for (; t + 4 < nk; t += 2) {  // lab\n"),
    ],
    "pstamps": [  # stamps inside the phases (the C park gives way: LDS is full with it)
        ("char smem[(DEFER && OUT != DT_F32 ? 10 : 8) * UNIT];", "char smem[8 * UNIT + 8192];"),
        ("  constexpr bool PARK = PAIRST;", "  constexpr bool PARK = false;  // lab: stamps"),
        ("  const bool g1 = wr == 1;  // wave-uniform (wave came through readfirstlane)",
         _PSTAMP_DEF),
        ("  wait_vm<0>();  // never leave an LDS-DMA in flight past the end of the workgroup",
         _STAMP_END),
        ("      stage_ab(same_tag, 1, BUF ^ 1, qa);\n      T4_LGKM0();\n",
         f"      stage_ab(same_tag, 1, BUF ^ 1, qa);\n      {_SB}\n      lab_stamp(1);\n      {_SB}\n"
         "      T4_LGKM0();\n"),
        ("      stage_ab(same_tag, 0, BUF, qb);\n      T4_LGKM0();\n",
         f"      stage_ab(same_tag, 0, BUF, qb);\n      {_SB}\n      lab_stamp(1);\n      {_SB}\n"
         "      T4_LGKM0();\n"),
        ("      mm(0, 0, Z);\n      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);\n",
         f"      mm(0, 0, Z);\n      {_SB}\n      lab_stamp(2);\n      {_SB}\n"
         "      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);\n"),
        ("      if constexpr (KIND == 1) mm(1, 1, false);\n"
         "      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);\n",
         f"      if constexpr (KIND == 1) mm(1, 1, false);\n      {_SB}\n      lab_stamp(2);\n"
         f"      {_SB}\n      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);\n"),
    ],
    "stamps": [  # (the C-park area gives way to the stamps: LDS is full with it)
        ("char smem[(DEFER && OUT != DT_F32 ? 10 : 8) * UNIT];", "char smem[8 * UNIT + 8192];"),
        ("  constexpr bool PARK = PAIRST;", "  constexpr bool PARK = false;  // lab: stamps"),
        ("  const bool g1 = wr == 1;  // wave-uniform (wave came through readfirstlane)",
         _STAMP_DEF),
        ("  wait_vm<0>();  // never leave an LDS-DMA in flight past the end of the workgroup",
         _STAMP_END),
    ],
}


REF_REV = os.environ.get("DDLB_LAB_REF", "HEAD")

# Variants measured and dropped against an earlier product kernel apply to the headers of that
# revision (the product moved on: the C park changed the code they patch); they rebuild exactly
# what was measured.
PINNED = {
    "behind": "2c4e4ca",   # r6_2
    "dmam": "38ab6ea",     # r6_3
    "dmam1": "38ab6ea",
    "lgkm_g0": "38ab6ea",  # r6_4
    "relax": "38ab6ea",    # r6_9
    "ring": "38ab6ea",     # r6_6
    "hold": "34f0106",     # r6_11
    "hold0": "b8b30bb",    # r6_16
    "dmafirst": "8c58daa",  # r6_18
    "dmamid": "8c58daa",
    "noprio": "8c58daa",    # r6_18, r6_19 (adopted for the 16-bit kernels)
    "lgkm0": "e2c6c5f",     # r6_21
    "prioload": "e2c6c5f",
    "krot": "e2c6c5f",      # r6_24
    "mrot": "e2c6c5f",      # r6_25
    "nocross": "e2c6c5f",   # r6_28 (adopted: stage_ab)
    "g1split": "cb084d4",   # r6_30 (adopted for the 16-bit flagship forms: SPLIT)
    "m0share": "fc1ce0f",   # r6_32 (exact, flat)
    "waitall": "fc1ce0f",   # r6_33 (MX spills)
    "unroll2": "d2e1ff0",   # r6_38 (flat)
}


def source(name: str, variant: str) -> str:
    """A header of csrc/gemm: from the working tree; for the ``ref`` variant from git revision
    ``DDLB_LAB_REF`` (default HEAD), so an edited kernel is timed against the committed one in
    the same process; for a PINNED variant from its revision."""
    rev = REF_REV if variant == "ref" else PINNED.get(variant)
    if rev is None:
        return open(os.path.join(CSRC, name)).read()
    return subprocess.run(["git", "-C", ROOT, "show", f"{rev}:csrc/gemm/{name}"],
                          capture_output=True, text=True, check=True).stdout


DIFFS = {  # variants kept as a diff against the product header (research/lab/<file>)
    "behind": "pt4_store_behind.diff",
    "ring": "pt4_a_ring.diff",
    "hold": "pt4_hold.diff",
    "hold0": "pt4_hold0.diff",
}


def _apply_diff(text: str, diff_name: str) -> str:
    import tempfile

    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, "csrc", "gemm"))
        with open(os.path.join(td, "csrc", "gemm", "gemm_kernels.h"), "w") as f:
            f.write(text)
        r = subprocess.run(["patch", "-p1", "-s", "-i", os.path.join(HERE, diff_name)],
                           cwd=td, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"{diff_name} does not apply: {r.stdout}{r.stderr}")
        return open(os.path.join(td, "csrc", "gemm", "gemm_kernels.h")).read()


def patched_header(variant: str) -> str:
    """The product header with the variant's substitutions applied inside the pt4 kernel's
    source (from its signature to the next kernel's); each pattern must occur exactly once."""
    src = source("gemm_kernels.h", variant)
    if variant in DIFFS:
        return _apply_diff(src, DIFFS[variant])
    i = src.index("void gemm_tn_pt4_kernel(")
    j = src.index("void gemm_tn_pt8_kernel(", i)
    body = src[i:j]
    pats = PATCHES[variant]
    if isinstance(pats, str):  # a combination of other variants' patches
        pats = [pt for v in pats.split("+") for pt in PATCHES[v]]
    for old, new in pats:
        n = body.count(old)
        if n != 1:
            raise RuntimeError(f"variant {variant}: pattern found {n} times: {old[:60]!r}")
        body = body.replace(old, new)
    return src[:i] + body + src[j:]


def build(variant: str, verbose: bool = False) -> str:
    """Compile one variant into research/lab/bin/pt4_<variant>.so (cached on the header text)."""
    import hashlib

    d = os.path.join(WORK, variant)
    os.makedirs(d, exist_ok=True)
    os.makedirs(BIN, exist_ok=True)
    for h in ("gemm.h", "tile_map.h"):
        with open(os.path.join(d, h), "w") as f:
            f.write(source(h, variant))
    text = patched_header(variant)
    with open(os.path.join(d, "gemm_kernels.h"), "w") as f:
        f.write(text)
    entry = open(os.path.join(HERE, "pt4_lab.hip")).read()
    dig = hashlib.sha256((text + entry + open(os.path.join(d, "gemm.h")).read() +
                          open(os.path.join(d, "tile_map.h")).read()).encode()).hexdigest()
    out = os.path.join(BIN, f"pt4_{variant}.so")
    stamp = out + ".sha256"
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read().strip() == dig:
        return out
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared",
           "--offload-arch=gfx950", f"-I{d}", os.path.join(HERE, "pt4_lab.hip"), "-o", out]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {variant}:\n{r.stderr[-4000:]}")
    with open(stamp, "w") as f:
        f.write(dig + "\n")
    return out


def main() -> int:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--variants", default=",".join(PATCHES))
    p.add_argument("--build-only", action="store_true")
    p.add_argument("--shapes", default="65536x1024x1024")
    p.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "mx"])
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--iters", type=int, default=40)
    p.add_argument("--vendor", action="store_true", help="also time F.linear (hipBLASLt)")
    p.add_argument("--stamp-report", action="store_true",
                   help="with the stamps variant: per-K-tile cycle profile of its last launch")
    a = p.parse_args()
    names = [v for v in a.variants.split(",") if v]
    if a.build_only:
        for v in names:
            print(v, build(v, verbose=True), flush=True)
        return 0
    import torch

    sys.path.insert(0, ROOT)
    from ddlb_amd.ops import gemm as G  # noqa: F401  (loads torch's HIP runtime first)

    libs = {}
    for v in names:
        lib = ctypes.CDLL(os.path.join(BIN, f"pt4_{v}.so"))
        lib.lab_pt4.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 + [ctypes.c_void_p] * 2
        lib.lab_pt4.restype = ctypes.c_int
        libs[v] = lib
    mx = a.dtype == "mx"
    dt = torch.float8_e4m3fn if mx else torch.bfloat16
    dbg = torch.zeros(1 << 22, dtype=torch.int32, device="cuda")
    for shp in a.shapes.split(","):
        M, N, K = (int(x) for x in shp.split("x"))
        A = (torch.rand((M, K), device="cuda") * 2 - 1).to(dt)
        W = (torch.rand((N, K), device="cuda") * 2 - 1).to(dt)
        out = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
        s = torch.cuda.current_stream().cuda_stream

        def launcher(v):
            lib = libs[v]

            def go():
                rc = lib.lab_pt4(A.data_ptr(), W.data_ptr(), out.data_ptr(), M, N, K, int(mx),
                                 dbg.data_ptr(), s)
                if rc != 0:
                    raise RuntimeError(f"{v}: lab_pt4 returned {rc}")
            return go

        fns = {v: launcher(v) for v in names}
        if a.vendor and not mx:
            fns["F.linear"] = lambda: torch.nn.functional.linear(A, W)
        exact = [v for v in fns if v in ("base", "ref", "stamps", "behind", "ring", "dmam", "dmam1",
                                         "lgkm_g0", "relax", "hold", "hold0", "dmafirst", "dmamid", "noprio", "lgkm0", "prioload", "pstamps", "krot", "mrot", "nocross", "g1split", "m0share", "waitall", "unroll2") or v.startswith(("aux", "stag"))]
        if exact:
            ref = A.float() @ W.float().t()
            bound = 2.0 ** -7 * float(ref.abs().max()) + K * 2.0 ** -12
            for v in exact:
                for rep in range(3):  # NaN-filled output, three launches: a race shows as NaN
                    out.fill_(float("nan"))
                    fns[v]()
                    torch.cuda.synchronize()
                    err = float(torch.nan_to_num((out.float() - ref).abs(),
                                                 nan=float("inf")).max())
                    if err > bound:
                        break
                print(f"{shp} {v} check: max|err| {err:.4g} (bound {bound:.4g}) "
                      f"{'ok' if err <= bound else 'FAIL'}", flush=True)
            del ref
        for _ in range(200):  # clock ramp
            fns[names[0]]()
        times = {k: [] for k in fns}
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for k, fn in fns.items():
                for _ in range(5):
                    fn()
                ev0.record()
                for _ in range(a.iters):
                    fn()
                ev1.record()
                torch.cuda.synchronize()
                times[k].append(ev0.elapsed_time(ev1) / a.iters)
        flop = 2.0 * M * N * K
        print(f"{shp} {a.dtype}: ms per launch, median / min over {a.rounds} rounds x "
              f"{a.iters}", flush=True)
        for k, ts in times.items():
            med = statistics.median(ts)
            print(f"  {k:10s} {med:.4f} / {min(ts):.4f}  ({flop / med / 1e9:.0f} TF)", flush=True)
        if a.stamp_report and "pstamps" in fns:
            dbg.zero_()
            for _ in range(20):
                fns["pstamps"]()
            torch.cuda.synchronize()
            pstamp_report(dbg.cpu())
        if a.stamp_report and "stamps" in fns:
            dbg.zero_()
            for _ in range(20):
                fns["stamps"]()
            torch.cuda.synchronize()
            stamp_report(dbg.cpu(), M, N, K, mx)
        del A, W, out
        torch.cuda.empty_cache()
    return 0


def pstamp_report(dbg, skip: int = 24) -> None:
    """Phase breakdown of one pstamps launch: per wave group, the median over workgroups and
    phases (stamps ``skip`` onwards: past the prologue) of each segment, in shader cycles. Load
    phase: 0 -> 1 reads + DMA issued, 1 -> 3 its waits (lgkmcnt, vmcnt), 3 -> 0 barrier; MFMA
    phase: 0 -> 2 MFMA issue, 2 -> 3 its waits, 3 -> 0 barrier."""
    import statistics

    import torch

    d = dbg.view(torch.int64).view(-1, 2, 512)
    nblk = int((d[:, 0, 2] > 0).sum())
    names = {(0, 1): "load: issue", (1, 3): "load: waits", (0, 2): "mfma: issue",
             (2, 3): "mfma: waits"}
    for g in range(2):
        seg = {}
        for b in range(nblk):
            n = min(int(d[b, g, 2]), 512)
            raw = [int(x) for x in d[b, g, 3:n]]
            st = [(x >> 4, x & 15) for x in raw]
            kind = None
            for i in range(max(skip, 1), len(st)):
                (t0, a), (t1, c) = st[i - 1], st[i]
                if a == 0 and c in (1, 2):
                    kind = "load" if c == 1 else "mfma"
                key = names.get((a, c))
                if key is None and (a, c) == (3, 0) and kind:
                    key = f"{kind}: barrier"
                if key:
                    seg.setdefault(key, []).append(t1 - t0)
        print(f"group {g}: median cycles per segment over {nblk} workgroups", flush=True)
        for key in ("load: issue", "load: waits", "load: barrier", "mfma: issue", "mfma: waits",
                    "mfma: barrier"):
            v = seg.get(key, [])
            if v:
                print(f"  {key:14s} {statistics.median(v):7.0f}  (p90 "
                      f"{sorted(v)[int(0.9 * (len(v) - 1))]:.0f}, n {len(v)})", flush=True)


def stamp_report(dbg, M: int, N: int, K: int, mx: bool) -> None:
    """Cycle profile of one stamps launch: per wave group, the median over workgroups of each
    barrier-to-barrier interval, summed per K-tile (4 barriers each), plus the clock."""
    import torch

    d = dbg.view(torch.int64).view(-1, 2, 512)
    nblk = int((d[:, 0, 2] > 0).sum())
    d = d[:nblk]
    wall_ns = (d[:, 0, 1] - d[:, 0, 0]).double() * 10.0  # s_memrealtime: 100 MHz
    n = int(d[:, :, 2].min())
    st = d[:, :, 3:n].double()
    cyc = st[:, :, -1] - st[:, :, 0]
    print(f"stamps: {nblk} workgroups, {n - 3} stamps per wave group, first -> last stamp "
          f"median {float(cyc.median()):.0f} cycles, workgroup wall median "
          f"{float(wall_ns.median()) / 1e3:.2f} us -> clock ~{float(cyc[:, 0].median()) / float(wall_ns.median()):.3f} GHz",
          flush=True)
    iv = st[:, :, 1:] - st[:, :, :-1]
    med = iv.median(dim=0).values  # [2, n-4]
    nk = K * (1 if mx else 2) // 128
    for g in range(2):
        row = med[g]
        print(f"group {g}: barrier intervals (median cycles over workgroups), {row.numel()} of "
              f"them; per K-tile sums of 4 (nk = {nk}):", flush=True)
        off = 1 if g == 0 else 2  # prologue barriers before the first K-tile's (g1 one more)
        body = row[off:]
        kt = [float(body[i:i + 4].sum()) for i in range(0, body.numel() - 3, 4)]
        for t0 in range(0, len(kt), nk):
            seg = kt[t0:t0 + nk]
            print(f"  tile {t0 // nk}: " + " ".join(f"{x:.0f}" for x in seg), flush=True)
        print("  first 12 intervals: " + " ".join(f"{float(x):.0f}" for x in row[:12]), flush=True)
        last = row[-12:]
        print("  last 12 intervals:  " + " ".join(f"{float(x):.0f}" for x in last), flush=True)


if __name__ == "__main__":
    sys.exit(main())
