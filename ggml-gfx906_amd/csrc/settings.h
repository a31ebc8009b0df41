// settings.h — every GGML_MI355X_* tuning / diagnostics knob, read from the environment ONCE
// into an immutable snapshot. The hot path reads fields of the snapshot (no getenv per call);
// tests and benches that switch a knob between calls re-read the environment through
// ggml_mi355x_reload_settings() (include/ggml-mi355x.h), which swaps in a new snapshot.
// Defaults are the product's behaviour; each field names its variable.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>

namespace mi355x {

struct Settings {
    // ---- mat-vec (ne11 <= 8)
    int rpw = 0;                  // GGML_MI355X_RPW: rows per wave (0 = pick_rpw's rule)
    int lpr = 0;                  // GGML_MI355X_LPR: 16 / 64 lanes per row (0 = by K)
    int64_t mmvq_wgs = 0;         // GGML_MI355X_MMVQ_WGS: target workgroups of a batched mat-vec (0 per type)
    int ring = 1;                 // GGML_MI355X_RING: 0 never the chunked-K kernel, 1 rule, 2 also 1 column
    int ring_pre = 1;             // GGML_MI355X_RING_PRE: 0 never pre-quantize, 1 from 4 columns, 2 from 2
    int ring_depth = 3;           // GGML_MI355X_RING_DEPTH: weight sets in flight (2 or 3)
    int64_t ring_wgs = 0;         // GGML_MI355X_RING_WGS: grid of the chunked kernel (0 = one round)
    int mma = -1;                 // GGML_MI355X_MMA: MFMA mat-vec from N columns (0 never, -1 rule)
    int mma_pair = -1;            // GGML_MI355X_MMA_PAIR: 0/1 force unpaired / paired steps (-1 plan)
    int mma_kh = 0;               // GGML_MI355X_MMA_KH: 1 / 2 force one / two K parts (0 plan)
    int mma_rt = 0;               // GGML_MI355X_MMA_RT: 1/2 row tiles per workgroup (0 plan)
    int solo = -1;                // GGML_MI355X_SOLO: single-wave kernel for one column (-1 rule, 0 off, 1 on, n rows per wave)
    // ---- mat-mat (ne11 > 8)
    int mmq_repack_min = 1 << 30; // GGML_MI355X_MMQ_REPACK_MIN: per-call repack from this many tokens (0 never)
    bool mmq_rp_all = false;      // GGML_MI355X_MMQ_RP_ALL=1: always read a caller's repacked copy
    int mmq8_tt = 0;              // GGML_MI355X_MMQ8_TT: 64 / 128 tokens per tile (0 = rule)
    int mmq8_tr = 0;              // GGML_MI355X_MMQ8_TR: 64 rows per tile with 64-token tiles
    int mmq8_ksplit = 0;          // GGML_MI355X_MMQ8_KSPLIT: split-K ways (0 = rule)
    bool mmq8_no_atomic = false;  // GGML_MI355X_MMQ8_ATOMIC=0: 2-way split-K through the reduce kernel
    int mmq8_sk = -1;             // GGML_MI355X_MMQ8_SK: stream-K 0 never / 1 whenever possible (-1 rule)
    int mmq_id_min = 64;          // GGML_MI355X_MMQ_ID_MIN: (slot, token) pairs for the grouped MUL_MAT_ID
    // ---- fused decode mat-vecs, GPT-2 engine, graph ops
    int fused_wgs = 256;          // GGML_MI355X_FUSED_WGS
    int fused_tall = 256;         // GGML_MI355X_FUSED_TALL
    int fused_lpr64_maxn = 1024;  // GGML_MI355X_FUSED_LPR64_MAXN
    bool attn_generic = false;    // GGML_MI355X_ATTN_GENERIC: the generic attention kernel (A/B)
    int gpt2_block = 1;           // GGML_MI355X_GPT2_BLOCK=0: the five-launch layer
    bool gpt2_embed_kernel = false; // GGML_MI355X_GPT2_EMBED_KERNEL: separate embedding launch
    // ---- backend (ggml plugin)
    bool debug = false;           // GGML_MI355X_DEBUG: log fusion / capture decisions
    bool fusion = true;           // GGML_MI355X_FUSION=0: no node fusion in graph_compute
    bool layer_fusion = true;     // GGML_MI355X_LAYER_FUSION=0: no whole-layer fusion
    bool graphs = true;           // GGML_MI355X_GRAPHS=0: no hipGraph capture
    int graph_max_updates = 4;    // GGML_MI355X_GRAPH_MAX_UPDATES
    int split_shards = 0;         // GGML_MI355X_SPLIT_SHARDS: virtual shards of the split buffer
    bool no_pinned = false;       // GGML_MI355X_NO_PINNED: no pinned host buffers
    int virtual_devices = 0;      // GGML_MI355X_VIRTUAL_DEVICES: plugin devices over the GPUs present
    // ---- diagnostics
    bool stamps = false;          // GGML_MI355X_STAMPS: per-workgroup s_memrealtime stamps
    int stamp_mv = -1;            // GGML_MI355X_STAMP_MV: which fused mat-vec of a step to stamp
    int diag = 0;                 // GGML_MI355X_DIAG (measurements; results wrong): bit 0 no activation loads,
                                  // bit 1 no weight loads, bit 8 (256) no mat-vec column pre-pass launch
};

// the current snapshot (the first call reads the environment)
const Settings &settings();
// re-read the environment into a new snapshot (earlier snapshots stay valid for their readers)
void reload_settings();

// Raise a kernel's dynamic-LDS limit to what the CU's 160 KiB leave beside its static arrays,
// once per (kernel, device). Not a stream operation; it fails inside a hipGraph capture (the
// launch then fails, the capture with it, and the caller's eager retry sets it).
struct LdsAttr {
    std::atomic<uint64_t> done{0};   // bit d: set on device d
};
hipError_t lds_attr_once(const void *kern, LdsAttr &flag);

}  // namespace mi355x
