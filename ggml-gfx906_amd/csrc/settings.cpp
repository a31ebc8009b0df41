// settings.cpp — the GGML_MI355X_* knobs of settings.h, read once per snapshot
#include "settings.h"

#include <cstdlib>
#include <mutex>

namespace mi355x {

static Settings load_settings() {
    auto i = [](const char *k, int d) {
        const char *e = getenv(k);
        return e ? atoi(e) : d;
    };
    auto l = [](const char *k, int64_t d) {
        const char *e = getenv(k);
        return e ? (int64_t)atoll(e) : d;
    };
    auto set = [](const char *k) { return getenv(k) != nullptr; };
    auto off = [](const char *k) {   // "=0" turns a default-on feature off
        const char *e = getenv(k);
        return e != nullptr && atoi(e) == 0;
    };
    Settings s;
    s.rpw = i("GGML_MI355X_RPW", 0);
    s.lpr = i("GGML_MI355X_LPR", 0);
    s.mmvq_wgs = l("GGML_MI355X_MMVQ_WGS", 0);
    s.ring = i("GGML_MI355X_RING", 1);
    s.ring_pre = i("GGML_MI355X_RING_PRE", 1);
    s.ring_depth = i("GGML_MI355X_RING_DEPTH", 3);
    s.ring_wgs = l("GGML_MI355X_RING_WGS", 0);
    s.mma = i("GGML_MI355X_MMA", -1);
    s.mma_pair = i("GGML_MI355X_MMA_PAIR", -1);
    s.mma_kh = i("GGML_MI355X_MMA_KH", 0);
    s.mma_rt = i("GGML_MI355X_MMA_RT", 0);
    s.solo = i("GGML_MI355X_SOLO", -1);
    s.mmq_repack_min = i("GGML_MI355X_MMQ_REPACK_MIN", 1 << 30);
    s.mmq_rp_all = i("GGML_MI355X_MMQ_RP_ALL", 0) == 1;
    s.mmq8_tt = i("GGML_MI355X_MMQ8_TT", 0);
    s.mmq8_tr = i("GGML_MI355X_MMQ8_TR", 0);
    s.mmq8_ksplit = i("GGML_MI355X_MMQ8_KSPLIT", 0);
    s.mmq8_no_atomic = off("GGML_MI355X_MMQ8_ATOMIC");
    s.mmq8_sk = i("GGML_MI355X_MMQ8_SK", -1);
    s.mmq_id_min = i("GGML_MI355X_MMQ_ID_MIN", 64);
    s.fused_wgs = i("GGML_MI355X_FUSED_WGS", 256);
    s.fused_tall = i("GGML_MI355X_FUSED_TALL", 256);
    s.fused_lpr64_maxn = i("GGML_MI355X_FUSED_LPR64_MAXN", 1024);
    s.attn_generic = set("GGML_MI355X_ATTN_GENERIC");
    s.gpt2_block = off("GGML_MI355X_GPT2_BLOCK") ? 0 : 1;
    s.gpt2_embed_kernel = set("GGML_MI355X_GPT2_EMBED_KERNEL");
    s.debug = set("GGML_MI355X_DEBUG");
    s.fusion = !off("GGML_MI355X_FUSION");
    s.layer_fusion = !off("GGML_MI355X_LAYER_FUSION");
    s.graphs = !off("GGML_MI355X_GRAPHS");
    s.graph_max_updates = i("GGML_MI355X_GRAPH_MAX_UPDATES", 4);
    s.split_shards = i("GGML_MI355X_SPLIT_SHARDS", 0);
    s.no_pinned = set("GGML_MI355X_NO_PINNED");
    s.virtual_devices = i("GGML_MI355X_VIRTUAL_DEVICES", 0);
    s.stamps = set("GGML_MI355X_STAMPS");
    s.stamp_mv = i("GGML_MI355X_STAMP_MV", -1);
    s.diag = i("GGML_MI355X_DIAG", 0);
    return s;
}

static std::atomic<const Settings *> g_settings{nullptr};
static std::mutex g_settings_mu;

const Settings &settings() {
    const Settings *p = g_settings.load(std::memory_order_acquire);
    if (p) return *p;
    std::lock_guard<std::mutex> lk(g_settings_mu);
    p = g_settings.load(std::memory_order_relaxed);
    if (!p) {
        p = new Settings(load_settings());
        g_settings.store(p, std::memory_order_release);
    }
    return *p;
}

void reload_settings() {
    std::lock_guard<std::mutex> lk(g_settings_mu);
    // the old snapshot is not freed: another thread may still be reading it (a few hundred
    // bytes per reload, and only tests and benches reload)
    g_settings.store(new Settings(load_settings()), std::memory_order_release);
}

hipError_t lds_attr_once(const void *kern, LdsAttr &flag) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        dev = 0;
    }
    const uint64_t bit = 1ull << (dev & 63);
    if (flag.done.load(std::memory_order_acquire) & bit) return hipSuccess;
    hipFuncAttributes fa{};
    hipError_t e = hipFuncGetAttributes(&fa, kern);
    if (e == hipSuccess)
        e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(160 * 1024 - fa.sharedSizeBytes));
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return e;
    }
    flag.done.fetch_or(bit, std::memory_order_acq_rel);
    return hipSuccess;
}

}  // namespace mi355x
