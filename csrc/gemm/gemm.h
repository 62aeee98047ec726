// Public interface of the CDNA4 MFMA GEMM (csrc/gemm/gemm_mfma.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ddlb {

// dtype codes shared with Python (ddlb_amd/ops/_dtypes.py)
enum DType : int { DT_F32 = 0, DT_F16 = 1, DT_BF16 = 2, DT_FP8 = 3, DT_F64 = 4, DT_U8 = 5 };
inline int dtype_size(int dt) {
  switch (dt) {
    case DT_F32: return 4;
    case DT_F16: case DT_BF16: return 2;
    case DT_FP8: case DT_U8: return 1;
    case DT_F64: return 8;
    default: return 0;
  }
}

// Codes 5 (pp256), 8 / 9 (p256 / p128), 13 / 14 (pi256 / pi256w4) and 15 (r256) belonged to
// kernel families retired in round 4 (no `auto` path reached them); they are refused.
enum Tile : int { TILE_AUTO = 0, TILE_256x256 = 1, TILE_256x128 = 2, TILE_128x256 = 3,
                  TILE_128x128 = 4, TILE_256x256_W4 = 6, TILE_256x128_W4 = 7,
                  TILE_I256 = 10, TILE_I128 = 11,    // I*: DMA interleaved into the MFMAs
                  TILE_I256W4 = 12,
                  TILE_T8 = 16,       // T8: 8-phase ping-pong, counted vmcnt (gemm_kernels.h)
                  TILE_PT8 = 17,      // PT8: persistent T8 (tiles streamed, C stores spread)
                  TILE_T4 = 18,       // T4: 2-phase ping-pong (32 MFMAs per section)
                  TILE_PT4 = 19 };    // PT4: persistent T4
// Every mode runs one of this file's hand-written kernels: vendor libraries (hipBLASLt through
// torch.matmul) are only the comparison baseline of the `pytorch` slot, never behind `native`.
enum GemmMode : int { GEMM_MODE_AUTO = 0, GEMM_MODE_GENERIC = 1, GEMM_MODE_MX = 2 };

// C[M,N] = A[M,K] * Bt[N,K]^T. Leading dimensions in ELEMENTS.
// Logical row i of A (and of C) lives at physical row (i / grp) * gstride + (i % grp).
struct GemmArgs {
  const void* a = nullptr;
  const void* b = nullptr;
  void* c = nullptr;
  int64_t lda = 0, ldb = 0, ldc = 0;
  int64_t a_grp = 0, a_gstride = 0;  // 0 -> identity
  int64_t c_grp = 0, c_gstride = 0;
  int M = 0, N = 0, K = 0;
  // Arrival-ordered consumption (p2p pipeline): optional
  const unsigned* flags = nullptr;  // flags[shard] >= epoch once shard's A rows have landed
  unsigned epoch = 0;
  const unsigned* epoch_ptr = nullptr;  // if set: the epoch is read here (hipGraph replay)
  int64_t flag_rows = 1;            // physical A rows per shard
  unsigned* timeout_word = nullptr; // set to 1 if a spin gave up
  unsigned spin_limit = 1u << 26;   // polls before a bounded spin gives up (~30 s on uncached flags)
  int tile_order = 0, nshards = 1, first_shard = 0;
  // Row blocks per producer (tile_order): shard index = producer * nsub + block; dispatch is
  // block-major across producers (block 0 of every producer, own first, then block 1, ...),
  // i.e. the order chunked pulls from all peers arrive in. nsub = 1: plain shard order.
  int nsub = 1;
  int reserve_cus = 0;              // flag-gated persistent GEMMs: CUs left free (see launch_pt4)
  int raster_g = 4;                 // m-blocks per raster group of tile_mn (tile_map.h)
  // In-kernel all-gather (flag-gated pt4 only): workgroups [0, ag_ctas) of the launch pull the
  // peers' row blocks of A over xGMI into A (the same rows), count each (producer, block)
  // segment's ag_parts pieces and set its flag when the last lands, and ACK each producer once
  // all its rows are read; the other workgroups run the gated GEMM. ag_tab (device, 2*np+2
  // entries, np = nshards / nsub producers): [src A of producer 0..np-1 | address of my ACK word
  // at producer 0..np-1 | READY words (ready[p] >= epoch: p's rows may be read) | counters
  // (nshards per-segment, then np per-producer; monotonic across runs) | with AG_WAIT_ACKS: my
  // ACK word written by producer 0..np-1 (entry of my own rank unused)].
  int ag_ctas = 0, ag_parts = 1, ag_rank = 0;
  int ag_mode = 0;                  // AgMode bits below
  const uint64_t* ag_tab = nullptr;
  int act = 0;                      // fused epilogue activation: ACT_* below
  // Direct-access A (optional): row block s of shard_rows rows starts at a_table[s] (device
  // array of addresses, e.g. the peers' IPC-mapped shards read straight over xGMI).
  const uint64_t* a_table = nullptr;
  int64_t shard_rows = 0;
  // Direct-store C (optional): row block s of c_shard_rows rows is written at c_table[s] (device
  // array of addresses, e.g. the peers' IPC-mapped receive slots: a reduce-scatter's partials
  // stored straight over xGMI by the GEMM epilogue). tile_order = 2 interleaves the shards.
  const uint64_t* c_table = nullptr;
  int64_t c_shard_rows = 0;
  // K-split (optional): ksplit slices of K columns each (K is the SLICE length; lda / ldb the
  // full rows); slice s reads A / B columns [s K, (s + 1) K) and writes its partial product at
  // c + s * M * ldc elements (the caller sums the partials). pt4 runs every (slice, tile) in one
  // launch; other kernels run the slices one after another.
  int ksplit = 1;
};
enum Act : int { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2, ACT_SILU = 3 };
// In-kernel all-gather variants (GemmArgs::ag_mode bits; 0 = write-through publication, 8 loads
// in flight per lane, system-scope acquire in the GEMM gate; the plan builders pick the default,
// ddlb_amd/parallel/algorithms.py AlgoConfig.ag_mode).
enum AgMode : int {
  AG_LEGACY_PUBLISH = 1,   // plain stores + agent release fence per unit (the first version)
  AG_AGENT_ACQUIRE = 2,    // the gated tiles acquire at agent scope (flags set by this launch)
  AG_DEEP_LOADS = 4,       // 16 loads in flight per lane instead of 8
  AG_FILL_ROUNDS = 8,      // grow ag_ctas while the GEMM's number of tile rounds stays the same
  AG_WAIT_ACKS = 16,       // copy workgroup 0 waits for every peer's ACK before the launch ends
                           // (ag_tab then has np more entries: my local ACK word per producer)
};

hipError_t gemm_launch(const GemmArgs& p, int din, int dout, int tile, int mode, hipStream_t s);
bool gemm_fast_path_ok(const GemmArgs& p, int din, int dout);
int choose_tile(int64_t M, int64_t N, int64_t K, int din);
int tile_rows(int tile);
int tile_cols(int tile);

}  // namespace ddlb
