/*
 * oracle/qref.c — CPU restatement of the reference's quantized MUL_MAT path.
 *
 * TEST INFRASTRUCTURE ONLY (see qref.h). Compiled with -ffp-contract=off so every float
 * expression rounds exactly as the reference's non-FMA ggml-base build does; the order of
 * every float operation below is the reference's order (that is the point of an oracle),
 * the code organisation is our own.
 *
 * Reference map (paths relative to the reference repo root):
 *   block layouts ............ src/ggml-common.h:170-344
 *   fp16 <-> fp32 ............ src/ggml-impl.h:358-405
 *   nearest_int .............. src/ggml-quants.c:444-449
 *   Q4_0 / Q8_0 / Q8_1 _ref .. src/ggml-quants.c:36-71, 199-257
 *   make_qx_quants ........... src/ggml-quants.c:451-518
 *   make_qkx2 / qkx3 / qp .... src/ggml-quants.c:622-701, 816-895, 899-969
 *   Q4_K / Q5_K / Q6_K ....... src/ggml-quants.c:1280-1463, 1467-1690, 1692-1891
 *   Q4_0 imatrix ............. src/ggml-quants.c:1893-1935;  Q8_0 chunk :2088-2093
 *   Q8_K ..................... src/ggml-quants.c:2555-2592
 *   dequantize_row_* ......... src/ggml-quants.c:307, 401, 1352, 1554, 1762
 *   ggml_quantize_chunk ...... src/ggml.c:6989-7060
 *   x86 quantize_row_q8_0 .... src/ggml-cpu/arch/x86/quants.c:290-360
 *   generic vec_dots ......... src/ggml-cpu/quants.c:115-149, 305-333, 550-623, 625-703, 705-758
 *   mul_mat / mul_mat_id ..... src/ggml-cpu/ggml-cpu.c:1112-1394, 1405-1655
 */
#include "qref.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <assert.h>
#include <pthread.h>
#include <unistd.h>

#define QK32  32
#define QKK   256
#define KSCALE 12

/* ------------------------------------------------------------------------------------ */
/* block layouts (byte-identical to src/ggml-common.h)                                   */
/* ------------------------------------------------------------------------------------ */
typedef struct { uint16_t d; uint8_t qs[16]; }                                  blk_q4_0;
typedef struct { uint16_t d; int8_t  qs[32]; }                                  blk_q8_0;
typedef struct { uint16_t d; uint16_t s; int8_t qs[32]; }                       blk_q8_1;
typedef struct { uint16_t d, dmin; uint8_t scales[KSCALE]; uint8_t qs[128]; }   blk_q4_K;
typedef struct { uint16_t d, dmin; uint8_t scales[KSCALE]; uint8_t qh[32]; uint8_t qs[128]; } blk_q5_K;
typedef struct { uint8_t ql[128]; uint8_t qh[64]; int8_t scales[16]; uint16_t d; } blk_q6_K;
typedef struct { float d; int8_t qs[256]; int16_t bsums[16]; }                  blk_q8_K;

_Static_assert(sizeof(blk_q4_0) == 18,  "q4_0");
_Static_assert(sizeof(blk_q8_0) == 34,  "q8_0");
_Static_assert(sizeof(blk_q8_1) == 36,  "q8_1");
_Static_assert(sizeof(blk_q4_K) == 144, "q4_K");
_Static_assert(sizeof(blk_q5_K) == 176, "q5_K");
_Static_assert(sizeof(blk_q6_K) == 210, "q6_K");
_Static_assert(sizeof(blk_q8_K) == 292, "q8_K");

#define IMIN(a, b) ((a) < (b) ? (a) : (b))
#define IMAX(a, b) ((a) > (b) ? (a) : (b))

int64_t qref_blck_size(int t) {
    switch (t) {
        case QREF_Q4_0: case QREF_Q8_0: case QREF_Q8_1: return QK32;
        case QREF_Q4_K: case QREF_Q5_K: case QREF_Q6_K: case QREF_Q8_K: return QKK;
        default: return 1;
    }
}

size_t qref_type_size(int t) {
    switch (t) {
        case QREF_F32:  return 4;
        case QREF_F16:  return 2;
        case QREF_I32:  return 4;
        case QREF_Q4_0: return sizeof(blk_q4_0);
        case QREF_Q8_0: return sizeof(blk_q8_0);
        case QREF_Q8_1: return sizeof(blk_q8_1);
        case QREF_Q4_K: return sizeof(blk_q4_K);
        case QREF_Q5_K: return sizeof(blk_q5_K);
        case QREF_Q6_K: return sizeof(blk_q6_K);
        case QREF_Q8_K: return sizeof(blk_q8_K);
        default: return 0;
    }
}

size_t qref_row_size(int t, int64_t ne) { return qref_type_size(t) * (size_t)(ne / qref_blck_size(t)); }

/* ggml-cpu type traits: which activation format each weight type dots against
 * (src/ggml-cpu/ggml-cpu.c:209-298) */
int qref_vec_dot_type(int t) {
    switch (t) {
        case QREF_Q4_0: case QREF_Q8_0: return QREF_Q8_0;
        case QREF_Q4_K: case QREF_Q5_K: case QREF_Q6_K: return QREF_Q8_K;
        case QREF_F32: return QREF_F32;
        default: return -1;
    }
}

/* ------------------------------------------------------------------------------------ */
/* scalar helpers                                                                        */
/* ------------------------------------------------------------------------------------ */
static inline uint32_t f_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float    f_from(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* IEEE binary16 -> binary32, exact (Maratyszcza's bit construction; ggml-impl.h:358-380) */
float qref_fp16_to_fp32(uint16_t h) {
    const uint32_t w      = (uint32_t)h << 16;
    const uint32_t sgn    = w & 0x80000000u;
    const uint32_t twice  = w + w;
    const float    norm   = f_from((twice >> 4) + (0xE0u << 23)) * 0x1.0p-112f;
    const float    denorm = f_from((twice >> 17) | (126u << 23)) - 0.5f;
    const uint32_t mag    = twice < (1u << 27) ? f_bits(denorm) : f_bits(norm);
    return f_from(sgn | mag);
}

/* binary32 -> binary16, round-to-nearest-even (ggml-impl.h:382-405) */
uint16_t qref_fp32_to_fp16(float f) {
    float base = (fabsf(f) * 0x1.0p+112f) * 0x1.0p-110f;
    const uint32_t w     = f_bits(f);
    const uint32_t twice = w + w;
    const uint32_t sgn   = w & 0x80000000u;
    uint32_t bias = twice & 0xFF000000u;
    if (bias < 0x71000000u) bias = 0x71000000u;
    base = f_from((bias >> 1) + 0x07800000u) + base;
    const uint32_t b    = f_bits(base);
    const uint32_t body = ((b >> 13) & 0x7C00u) + (b & 0x0FFFu);
    return (uint16_t)((sgn >> 16) | (twice > 0xFF000000u ? 0x7E00u : body));
}

#define H2F(h) qref_fp16_to_fp32(h)
#define F2H(f) qref_fp32_to_fp16(f)

/* round-half-even to int through the 1.5*2^23 magic (ggml-quants.c:444-449) */
static inline int rne_int(float v) {
    const float t = v + 12582912.f;
    return (int)(f_bits(t) & 0x007fffffu) - 0x00400000;
}

void qref_fill_uniform(float *dst, int64_t n, uint64_t seed, float lo, float hi) {
    for (int64_t i = 0; i < n; ++i) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const float u = (float)(z >> 40) * 0x1.0p-24f;   /* [0,1), 24 random bits, exact */
        dst[i] = lo + (hi - lo) * u;
    }
}

/* ------------------------------------------------------------------------------------ */
/* Q4_0 / Q8_0 / Q8_1 reference quantizers                                               */
/* ------------------------------------------------------------------------------------ */

/* ggml-quants.c:36-71 — signed max -> d = max/-8, q = min(15, (int8)(x/d + 8.5)) */
static void q4_0_from_f32(const float *x, blk_q4_0 *y, int64_t nblk) {
    for (int64_t b = 0; b < nblk; ++b, x += QK32) {
        float big = 0.0f, signed_big = 0.0f;
        for (int j = 0; j < QK32; ++j) {
            if (big < fabsf(x[j])) { big = fabsf(x[j]); signed_big = x[j]; }
        }
        const float d  = signed_big / -8;
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = F2H(d);
        for (int j = 0; j < 16; ++j) {
            const uint8_t lo = (uint8_t)IMIN(15, (int8_t)(x[j] * id + 8.5f));
            const uint8_t hi = (uint8_t)IMIN(15, (int8_t)(x[j + 16] * id + 8.5f));
            y[b].qs[j] = (uint8_t)(lo | (hi << 4));
        }
    }
}

/* ggml-quants.c:199-222 — d = amax/127, q = roundf(x*id) */
static void q8_0_from_f32(const float *x, blk_q8_0 *y, int64_t nblk) {
    for (int64_t b = 0; b < nblk; ++b, x += QK32) {
        float amax = 0.0f;
        for (int j = 0; j < QK32; ++j) amax = amax > fabsf(x[j]) ? amax : fabsf(x[j]);
        const float d  = amax / ((1 << 7) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = F2H(d);
        for (int j = 0; j < QK32; ++j) y[b].qs[j] = (int8_t)roundf(x[j] * id);
    }
}

/* ggml-quants.c:225-257 — as Q8_0 plus s = fp16(d * sum(q)) */
static void q8_1_from_f32(const float *x, blk_q8_1 *y, int64_t nblk) {
    for (int64_t b = 0; b < nblk; ++b, x += QK32) {
        float amax = 0.0f;
        for (int j = 0; j < QK32; ++j) amax = amax > fabsf(x[j]) ? amax : fabsf(x[j]);
        const float d  = amax / ((1 << 7) - 1);
        const float id = d ? 1.0f / d : 0.0f;
        y[b].d = F2H(d);
        int sum = 0;
        for (int j = 0; j < 16; ++j) {
            y[b].qs[j]      = (int8_t)roundf(x[j] * id);
            y[b].qs[j + 16] = (int8_t)roundf(x[j + 16] * id);
            sum += y[b].qs[j] + y[b].qs[j + 16];
        }
        y[b].s = F2H(sum * d);
    }
}

/* arch/x86/quants.c:290-360 (AVX2 path actually run by ggml-cpu on x86):
 * d = amax/127 stored as fp16, multiplier 127/amax, round-to-nearest-even */
static void q8_0_from_f32_x86(const float *x, blk_q8_0 *y, int64_t nblk) {
    for (int64_t b = 0; b < nblk; ++b, x += QK32) {
        float amax = 0.0f;
        for (int j = 0; j < QK32; ++j) if (fabsf(x[j]) > amax) amax = fabsf(x[j]);
        const float d   = amax / 127.f;
        const float mul = amax != 0.0f ? 127.f / amax : 0.0f;
        y[b].d = F2H(d);
        for (int j = 0; j < QK32; ++j) y[b].qs[j] = (int8_t)(int)rintf(x[j] * mul);
    }
}

/* ggml-quants.c:2555-2592 — Q8_K: signed max, iscale = -127/max, bsums per 16 */
static void q8_K_from_f32(const float *x, blk_q8_K *y, int64_t nblk) {
    for (int64_t b = 0; b < nblk; ++b, x += QKK) {
        float amax = 0, smax = 0;
        for (int j = 0; j < QKK; ++j) {
            if (fabsf(x[j]) > amax) { amax = fabsf(x[j]); smax = x[j]; }
        }
        if (!amax) {
            y[b].d = 0;
            memset(y[b].qs, 0, QKK);
            /* bsums are left as-is by the reference; zero them for determinism */
            memset(y[b].bsums, 0, sizeof(y[b].bsums));
            continue;
        }
        const float iscale = -127.f / smax;
        for (int j = 0; j < QKK; ++j) y[b].qs[j] = (int8_t)IMIN(127, rne_int(iscale * x[j]));
        for (int g = 0; g < 16; ++g) {
            int s = 0;
            for (int i = 0; i < 16; ++i) s += y[b].qs[16 * g + i];
            y[b].bsums[g] = (int16_t)s;
        }
        y[b].d = 1 / iscale;
    }
}

/* ------------------------------------------------------------------------------------ */
/* k-quant search helpers                                                                */
/* ------------------------------------------------------------------------------------ */

/* weight function of make_qx_quants (ggml-quants.c:451-518) */
static inline float qx_weight(const float *qw, const float *x, int i, int rmse_type) {
    if (qw) return qw[i];
    switch (rmse_type) {
        case 1:  return x[i] * x[i];
        case 2:  return 1;
        case 3:  return fabsf(x[i]);
        default: return sqrtf(fabsf(x[i]));
    }
}

/* symmetric search: 19 candidate scales around -nmax/max; L in [0, 2*nmax) */
static float search_symmetric(int n, int nmax, const float *x, int8_t *L, int rmse_type, const float *qw) {
    float amax = 0, smax = 0;
    for (int i = 0; i < n; ++i) {
        if (fabsf(x[i]) > amax) { amax = fabsf(x[i]); smax = x[i]; }
    }
    if (amax < 1e-15f) {
        memset(L, 0, (size_t)n);
        return 0.f;
    }
    float iscale = -nmax / smax;
    if (rmse_type == 0) {
        for (int i = 0; i < n; ++i) L[i] = (int8_t)(nmax + IMAX(-nmax, IMIN(nmax - 1, rne_int(iscale * x[i]))));
        return 1 / iscale;
    }
    int early = 0;
    if (rmse_type < 0) { rmse_type = -rmse_type; early = 1; }
    float slx = 0, sl2 = 0;
    for (int i = 0; i < n; ++i) {
        const int l = IMAX(-nmax, IMIN(nmax - 1, rne_int(iscale * x[i])));
        L[i] = (int8_t)(l + nmax);
        const float w = qx_weight(qw, x, i, rmse_type);
        slx += w * x[i] * l;
        sl2 += w * l * l;
    }
    float scale = sl2 ? slx / sl2 : 0.0f;
    if (early) return sl2 > 0 ? 0.5f * (scale + 1 / iscale) : 1 / iscale;
    float best = scale * slx;
    for (int step = -9; step <= 9; ++step) {
        if (step == 0) continue;
        iscale = -(nmax + 0.1f * step) / smax;
        slx = sl2 = 0;
        for (int i = 0; i < n; ++i) {
            const int l = IMAX(-nmax, IMIN(nmax - 1, rne_int(iscale * x[i])));
            const float w = qx_weight(qw, x, i, rmse_type);
            slx += w * x[i] * l;
            sl2 += w * l * l;
        }
        if (sl2 > 0 && slx * slx > best * sl2) {
            for (int i = 0; i < n; ++i) L[i] = (int8_t)(nmax + IMAX(-nmax, IMIN(nmax - 1, rne_int(iscale * x[i]))));
            scale = slx / sl2;
            best  = scale * slx;
        }
    }
    return scale;
}

/* asymmetric (scale, min) grid search — make_qkx2_quants (weights given) and make_qkx3_quants
 * (weights may be NULL -> x^2) share this body; they differ only in the degenerate-range test
 * (qkx2: max == min, qkx3: max <= min) and the memset vs loop (same result). */
static float search_affine(int n, int nmax, const float *x, const float *weights, uint8_t *L,
                           float *the_min, uint8_t *Laux, float rmin, float rdelta, int nstep,
                           int use_mad, int strict_le) {
#define W_AT(i) (weights ? weights[(i)] : x[(i)] * x[(i)])
    float lo = x[0], hi = x[0];
    float sum_w = W_AT(0);
    float sum_x = sum_w * x[0];
    for (int i = 1; i < n; ++i) {
        if (x[i] < lo) lo = x[i];
        if (x[i] > hi) hi = x[i];
        const float w = W_AT(i);
        sum_w += w;
        sum_x += w * x[i];
    }
    if (lo > 0) lo = 0;
    if (strict_le ? (hi <= lo) : (hi == lo)) {
        memset(L, 0, (size_t)n);
        *the_min = -lo;
        return 0.f;
    }
    float iscale = nmax / (hi - lo);
    float scale  = 1 / iscale;
    float best_err = 0;
    for (int i = 0; i < n; ++i) {
        const int l = rne_int(iscale * (x[i] - lo));
        L[i] = (uint8_t)IMAX(0, IMIN(nmax, l));
        float diff = scale * L[i] + lo - x[i];
        diff = use_mad ? fabsf(diff) : diff * diff;
        best_err += W_AT(i) * diff;
    }
    if (nstep < 1) {
        *the_min = -lo;
        return scale;
    }
    for (int step = 0; step <= nstep; ++step) {
        iscale = (rmin + rdelta * step + nmax) / (hi - lo);
        float s_l = 0, s_l2 = 0, s_xl = 0;
        for (int i = 0; i < n; ++i) {
            const int l = IMAX(0, IMIN(nmax, rne_int(iscale * (x[i] - lo))));
            Laux[i] = (uint8_t)l;
            const float w = W_AT(i);
            s_l  += w * l;
            s_l2 += w * l * l;
            s_xl += w * l * x[i];
        }
        const float D = sum_w * s_l2 - s_l * s_l;
        if (D > 0) {
            float this_scale = (sum_w * s_xl - sum_x * s_l) / D;
            float this_min   = (s_l2 * sum_x - s_l * s_xl) / D;
            if (this_min > 0) {
                this_min   = 0;
                this_scale = s_xl / s_l2;
            }
            float err = 0;
            for (int i = 0; i < n; ++i) {
                float diff = this_scale * Laux[i] + this_min - x[i];
                diff = use_mad ? fabsf(diff) : diff * diff;
                err += W_AT(i) * diff;
            }
            if (err < best_err) {
                memcpy(L, Laux, (size_t)n);
                best_err = err;
                scale    = this_scale;
                lo       = this_min;
            }
        }
    }
    *the_min = -lo;
    return scale;
#undef W_AT
}

/* make_qp_quants (ggml-quants.c:899-969): positive-only quantization of the sub-block scales */
static float search_positive(int n, int nmax, const float *x, uint8_t *L, const float *qw) {
    float top = 0;
    for (int i = 0; i < n; ++i) top = top > x[i] ? top : x[i];
    if (top < 1e-15f) {
        memset(L, 0, (size_t)n);
        return 0.f;
    }
    float iscale = nmax / top;
    for (int i = 0; i < n; ++i) L[i] = (uint8_t)rne_int(iscale * x[i]);
    const float scale0 = 1 / iscale;
    float best_mse = 0;
    for (int i = 0; i < n; ++i) {
        const float diff = x[i] - scale0 * L[i];
        best_mse += qw[i] * diff * diff;
    }
    for (int step = -4; step <= 4; ++step) {
        if (step == 0) continue;
        const float is_try = (0.1f * step + nmax) / top;
        const float sc_try = 1 / is_try;
        float mse = 0;
        for (int i = 0; i < n; ++i) {
            const int l = IMIN(nmax, rne_int(is_try * x[i]));
            const float diff = x[i] - sc_try * l;
            mse += qw[i] * diff * diff;
        }
        if (mse < best_mse) {
            best_mse = mse;
            iscale   = is_try;
        }
    }
    float slx = 0, sl2 = 0;
    for (int i = 0; i < n; ++i) {
        const int l = IMIN(nmax, rne_int(iscale * x[i]));
        L[i] = (uint8_t)l;
        slx += qw[i] * x[i] * l;
        sl2 += qw[i] * l * l;
    }
    for (int pass = 0; pass < 5; ++pass) {
        int changed = 0;
        for (int i = 0; i < n; ++i) {
            const float w = qw[i];
            float s1 = slx - w * x[i] * L[i];
            float s2 = sl2 - w * L[i] * L[i];
            if (s1 > 0 && s2 > 0) {
                const int nl = IMIN(nmax, rne_int(x[i] * s2 / s1));
                if (nl != L[i]) {
                    s1 += w * x[i] * nl;
                    s2 += w * nl * nl;
                    if (s1 * s1 * sl2 > slx * slx * s2) {
                        L[i] = (uint8_t)nl;
                        slx = s1;
                        sl2 = s2;
                        ++changed;
                    }
                }
            }
        }
        if (!changed) break;
    }
    return sl2 > 0.0f ? slx / sl2 : 0.0f;
}

/* 6-bit (scale, min) packing of Q4_K/Q5_K (ggml-quants.c:1317-1328) and its inverse
 * get_scale_min_k4 (ggml-quants.c:703-710) */
static void pack_scale_min(uint8_t *sc12, int j, uint8_t ls, uint8_t lm) {
    if (j < 4) {
        sc12[j]     = ls;
        sc12[j + 4] = lm;
    } else {
        sc12[j + 4]  = (uint8_t)((ls & 0xF) | ((lm & 0xF) << 4));
        sc12[j - 4] |= (uint8_t)((ls >> 4) << 6);
        sc12[j]     |= (uint8_t)((lm >> 4) << 6);
    }
}

static void unpack_scale_min(const uint8_t *sc12, int j, uint8_t *s, uint8_t *m) {
    if (j < 4) {
        *s = sc12[j] & 63;
        *m = sc12[j + 4] & 63;
    } else {
        *s = (uint8_t)((sc12[j + 4] & 0xF) | ((sc12[j - 4] >> 6) << 4));
        *m = (uint8_t)((sc12[j + 4] >> 4) | ((sc12[j] >> 6) << 4));
    }
}

/* ------------------------------------------------------------------------------------ */
/* Q4_K / Q5_K (shared 8x32 sub-block structure)                                          */
/* ------------------------------------------------------------------------------------ */

/* re-quantize each 32-run against the already-packed (d, dmin, scales): ggml-quants.c:1333-1344 */
static void kquant_levels(const float *x, const uint8_t *sc12, uint16_t hd, uint16_t hdmin,
                          int qmax, uint8_t *L) {
    for (int j = 0; j < 8; ++j) {
        uint8_t s, m;
        unpack_scale_min(sc12, j, &s, &m);
        const float d = H2F(hd) * s;
        if (!d) continue;
        const float dm = H2F(hdmin) * m;
        for (int i = 0; i < 32; ++i) {
            const int l = rne_int((x[32 * j + i] + dm) / d);
            L[32 * j + i] = (uint8_t)IMAX(0, IMIN(qmax, l));
        }
    }
}

/* _ref flavour (ggml-quants.c:1280-1350 for Q4_K, 1467-1552 for Q5_K) */
static void k45_ref_superblock(const float *x, uint8_t *sc12, uint16_t *hd, uint16_t *hdmin,
                               uint8_t *L, int qmax, float rmin, int nstep) {
    float scales[8], mins[8], w[32];
    uint8_t Laux[32];
    float max_scale = 0, max_min = 0;
    for (int j = 0; j < 8; ++j) {
        float sx2 = 0;
        for (int l = 0; l < 32; ++l) sx2 += x[32 * j + l] * x[32 * j + l];
        const float av = sqrtf(sx2 / 32);
        for (int l = 0; l < 32; ++l) w[l] = av + fabsf(x[32 * j + l]);
        scales[j] = search_affine(32, qmax, x + 32 * j, w, L + 32 * j, &mins[j], Laux, rmin, 0.1f, nstep, 0, 0);
        if (scales[j] > max_scale) max_scale = scales[j];
        if (mins[j] > max_min) max_min = mins[j];
    }
    const float inv_s = max_scale > 0 ? 63.f / max_scale : 0.f;
    const float inv_m = max_min > 0 ? 63.f / max_min : 0.f;
    memset(sc12, 0, KSCALE);
    for (int j = 0; j < 8; ++j) {
        uint8_t ls = (uint8_t)rne_int(inv_s * scales[j]);
        uint8_t lm = (uint8_t)rne_int(inv_m * mins[j]);
        ls = ls < 63 ? ls : 63;
        lm = lm < 63 ? lm : 63;
        pack_scale_min(sc12, j, ls, lm);
    }
    *hd    = F2H(max_scale / 63.f);
    *hdmin = F2H(max_min / 63.f);
    kquant_levels(x, sc12, *hd, *hdmin, qmax, L);
}

/* imatrix flavour (ggml-quants.c:1376-1447 for Q4_K, 1581-1672 for Q5_K) */
static void k45_imx_superblock(const float *x, const float *qw, uint8_t *sc12, uint16_t *hd,
                               uint16_t *hdmin, uint8_t *L, int qmax) {
    float scales[8], mins[8], sw[8], w[32];
    uint8_t Laux[32], Ls[8], Lm[8];
    float sx2 = 0;
    for (int l = 0; l < QKK; ++l) sx2 += x[l] * x[l];
    const float sigma2 = 2 * sx2 / QKK;
    const float av = sqrtf(sigma2);
    for (int j = 0; j < 8; ++j) {
        if (qw) {
            const float *q = qw + 32 * j;
            for (int l = 0; l < 32; ++l) w[l] = q[l] * sqrtf(sigma2 + x[32 * j + l] * x[32 * j + l]);
        } else {
            for (int l = 0; l < 32; ++l) w[l] = av + fabsf(x[32 * j + l]);
        }
        float s = 0;
        for (int l = 0; l < 32; ++l) s += w[l];
        sw[j] = s;
        scales[j] = search_affine(32, qmax, x + 32 * j, w, L + 32 * j, &mins[j], Laux, -0.9f, 0.05f, 36, 0, 1);
    }
    const float d_blk = search_positive(8, 63, scales, Ls, sw);
    const float m_blk = search_positive(8, 63, mins, Lm, sw);
    memset(sc12, 0, KSCALE);
    for (int j = 0; j < 8; ++j) {
        const uint8_t ls = Ls[j] < 63 ? Ls[j] : 63;
        const uint8_t lm = Lm[j] < 63 ? Lm[j] : 63;
        pack_scale_min(sc12, j, ls, lm);
    }
    *hd    = F2H(d_blk);
    *hdmin = F2H(m_blk);
    kquant_levels(x, sc12, *hd, *hdmin, qmax, L);
}

static void q4_K_pack_levels(blk_q4_K *y, const uint8_t *L) {
    for (int c = 0; c < 4; ++c)
        for (int l = 0; l < 32; ++l) y->qs[32 * c + l] = (uint8_t)(L[64 * c + l] | (L[64 * c + 32 + l] << 4));
}

static void q5_K_pack_levels(blk_q5_K *y, const uint8_t *L) {
    memset(y->qh, 0, 32);
    for (int c = 0; c < 4; ++c) {
        for (int l = 0; l < 32; ++l) {
            int a = L[64 * c + l], b = L[64 * c + 32 + l];
            if (a > 15) { a -= 16; y->qh[l] |= (uint8_t)(1u << (2 * c)); }
            if (b > 15) { b -= 16; y->qh[l] |= (uint8_t)(2u << (2 * c)); }
            y->qs[32 * c + l] = (uint8_t)(a | (b << 4));
        }
    }
}

static void q4_K_from_f32(const float *x, blk_q4_K *y, int64_t nblk, const float *qw, int imx) {
    uint8_t L[QKK];
    for (int64_t b = 0; b < nblk; ++b, x += QKK) {
        if (imx) k45_imx_superblock(x, qw ? qw + QKK * b : NULL, y[b].scales, &y[b].d, &y[b].dmin, L, 15);
        else     k45_ref_superblock(x, y[b].scales, &y[b].d, &y[b].dmin, L, 15, -1.f, 20);
        q4_K_pack_levels(&y[b], L);
    }
}

static void q5_K_from_f32(const float *x, blk_q5_K *y, int64_t nblk, const float *qw, int imx) {
    uint8_t L[QKK];
    for (int64_t b = 0; b < nblk; ++b, x += QKK) {
        if (imx) k45_imx_superblock(x, qw ? qw + QKK * b : NULL, y[b].scales, &y[b].d, &y[b].dmin, L, 31);
        else     k45_ref_superblock(x, y[b].scales, &y[b].d, &y[b].dmin, L, 31, -0.5f, 15);
        q5_K_pack_levels(&y[b], L);
    }
}

/* ------------------------------------------------------------------------------------ */
/* Q6_K (16x16 sub-blocks, int8 scales) — ggml-quants.c:1692-1760 / 1793-1875             */
/* ------------------------------------------------------------------------------------ */
static void q6_K_from_f32(const float *x, blk_q6_K *y, int64_t nblk, const float *qw) {
    int8_t L[QKK];
    float scales[16];
    for (int64_t b = 0; b < nblk; ++b, x += QKK) {
        float max_scale = 0, max_abs = 0;
        for (int g = 0; g < 16; ++g) {
            const float s = search_symmetric(16, 32, x + 16 * g, L + 16 * g, 1, qw ? qw + QKK * b + 16 * g : NULL);
            scales[g] = s;
            if (fabsf(s) > max_abs) { max_abs = fabsf(s); max_scale = s; }
        }
        if (max_abs < 1e-15f) {
            memset(&y[b], 0, sizeof(y[b]));
            y[b].d = F2H(0.f);
            continue;
        }
        const float iscale = -128.f / max_scale;
        y[b].d = F2H(1 / iscale);
        for (int g = 0; g < 16; ++g) y[b].scales[g] = (int8_t)IMIN(127, rne_int(iscale * scales[g]));
        for (int g = 0; g < 16; ++g) {
            const float d = H2F(y[b].d) * y[b].scales[g];
            if (!d) continue;
            for (int i = 0; i < 16; ++i) {
                const int l = IMAX(-32, IMIN(31, rne_int(x[16 * g + i] / d)));
                L[16 * g + i] = (int8_t)(l + 32);
            }
        }
        for (int h = 0; h < 2; ++h) {
            const int8_t *Lh = L + 128 * h;
            uint8_t *ql = y[b].ql + 64 * h;
            uint8_t *qh = y[b].qh + 32 * h;
            for (int l = 0; l < 32; ++l) {
                const uint8_t v0 = (uint8_t)Lh[l], v1 = (uint8_t)Lh[l + 32], v2 = (uint8_t)Lh[l + 64], v3 = (uint8_t)Lh[l + 96];
                ql[l]      = (uint8_t)((v0 & 0xF) | ((v2 & 0xF) << 4));
                ql[l + 32] = (uint8_t)((v1 & 0xF) | ((v3 & 0xF) << 4));
                qh[l]      = (uint8_t)((v0 >> 4) | ((v1 >> 4) << 2) | ((v2 >> 4) << 4) | ((v3 >> 4) << 6));
            }
        }
    }
}

/* Q4_0 with importance weights (ggml-quants.c:1893-1919); sigma2 over the whole row */
static void q4_0_from_f32_imx(const float *x, blk_q4_0 *y, int64_t n_per_row, const float *qw) {
    float sx2 = 0;
    for (int64_t j = 0; j < n_per_row; ++j) sx2 += x[j] * x[j];
    const float sigma2 = sx2 / n_per_row;
    float w[QK32];
    int8_t L[QK32];
    for (int64_t b = 0; b < n_per_row / QK32; ++b) {
        const float *xb = x + QK32 * b, *q = qw + QK32 * b;
        for (int j = 0; j < QK32; ++j) w[j] = q[j] * sqrtf(sigma2 + xb[j] * xb[j]);
        const float d = search_symmetric(QK32, 8, xb, L, 1, w);
        y[b].d = F2H(d);
        for (int j = 0; j < 16; ++j) y[b].qs[j] = (uint8_t)(L[j] | (L[j + 16] << 4));
    }
}

void qref_quantize_row_ref(int type, const float *x, void *y, int64_t k) {
    switch (type) {
        case QREF_Q4_0: q4_0_from_f32(x, (blk_q4_0 *)y, k / QK32); break;
        case QREF_Q8_0: q8_0_from_f32(x, (blk_q8_0 *)y, k / QK32); break;
        case QREF_Q8_1: q8_1_from_f32(x, (blk_q8_1 *)y, k / QK32); break;
        case QREF_Q4_K: q4_K_from_f32(x, (blk_q4_K *)y, k / QKK, NULL, 0); break;
        case QREF_Q5_K: q5_K_from_f32(x, (blk_q5_K *)y, k / QKK, NULL, 0); break;
        case QREF_Q6_K: q6_K_from_f32(x, (blk_q6_K *)y, k / QKK, NULL); break;
        case QREF_Q8_K: q8_K_from_f32(x, (blk_q8_K *)y, k / QKK); break;
        default: abort();
    }
}

/* ggml_quantize_chunk (ggml.c:6989-7060) + per-type dispatchers quantize_q* */
size_t qref_quantize_chunk(int type, const float *src, void *dst, int64_t start, int64_t nrows,
                           int64_t n_per_row, const float *imatrix) {
    const size_t rs = qref_row_size(type, n_per_row);
    const float *x  = src + start;
    uint8_t *out    = (uint8_t *)dst + (size_t)(start / n_per_row) * rs;
    if (!imatrix || type == QREF_Q8_0) {
        qref_quantize_row_ref(type, x, out, nrows * n_per_row);
        return (size_t)nrows * rs;
    }
    for (int64_t r = 0; r < nrows; ++r, x += n_per_row, out += rs) {
        switch (type) {
            case QREF_Q4_0: q4_0_from_f32_imx(x, (blk_q4_0 *)out, n_per_row, imatrix); break;
            case QREF_Q4_K: q4_K_from_f32(x, (blk_q4_K *)out, n_per_row / QKK, imatrix, 1); break;
            case QREF_Q5_K: q5_K_from_f32(x, (blk_q5_K *)out, n_per_row / QKK, imatrix, 1); break;
            case QREF_Q6_K: q6_K_from_f32(x, (blk_q6_K *)out, n_per_row / QKK, imatrix); break;
            default: abort();
        }
    }
    return (size_t)nrows * rs;
}

/* ------------------------------------------------------------------------------------ */
/* dequantization (bit-exact targets for the device dequant kernels)                     */
/* ------------------------------------------------------------------------------------ */
void qref_dequantize_row(int type, const void *vx, float *y, int64_t k) {
    switch (type) {
    case QREF_Q4_0: {                                   /* ggml-quants.c:307-323 */
        const blk_q4_0 *x = (const blk_q4_0 *)vx;
        for (int64_t b = 0; b < k / QK32; ++b, y += QK32) {
            const float d = H2F(x[b].d);
            for (int j = 0; j < 16; ++j) {
                y[j]      = ((x[b].qs[j] & 0x0F) - 8) * d;
                y[j + 16] = ((x[b].qs[j] >> 4) - 8) * d;
            }
        }
    } break;
    case QREF_Q8_0: {                                   /* ggml-quants.c:401-415 */
        const blk_q8_0 *x = (const blk_q8_0 *)vx;
        for (int64_t b = 0; b < k / QK32; ++b, y += QK32) {
            const float d = H2F(x[b].d);
            for (int j = 0; j < QK32; ++j) y[j] = x[b].qs[j] * d;
        }
    } break;
    case QREF_Q4_K: {                                   /* ggml-quants.c:1352-1374 */
        const blk_q4_K *x = (const blk_q4_K *)vx;
        for (int64_t b = 0; b < k / QKK; ++b) {
            const float d = H2F(x[b].d), mn = H2F(x[b].dmin);
            for (int c = 0; c < 4; ++c) {
                uint8_t s, m;
                unpack_scale_min(x[b].scales, 2 * c, &s, &m);
                const float d1 = d * s, m1 = mn * m;
                unpack_scale_min(x[b].scales, 2 * c + 1, &s, &m);
                const float d2 = d * s, m2 = mn * m;
                const uint8_t *q = x[b].qs + 32 * c;
                for (int l = 0; l < 32; ++l) *y++ = d1 * (q[l] & 0xF) - m1;
                for (int l = 0; l < 32; ++l) *y++ = d2 * (q[l] >> 4) - m2;
            }
        }
    } break;
    case QREF_Q5_K: {                                   /* ggml-quants.c:1554-1579 */
        const blk_q5_K *x = (const blk_q5_K *)vx;
        for (int64_t b = 0; b < k / QKK; ++b) {
            const float d = H2F(x[b].d), mn = H2F(x[b].dmin);
            for (int c = 0; c < 4; ++c) {
                uint8_t s, m;
                unpack_scale_min(x[b].scales, 2 * c, &s, &m);
                const float d1 = d * s, m1 = mn * m;
                unpack_scale_min(x[b].scales, 2 * c + 1, &s, &m);
                const float d2 = d * s, m2 = mn * m;
                const uint8_t *q = x[b].qs + 32 * c;
                const uint8_t u1 = (uint8_t)(1u << (2 * c)), u2 = (uint8_t)(2u << (2 * c));
                for (int l = 0; l < 32; ++l) *y++ = d1 * ((q[l] & 0xF) + (x[b].qh[l] & u1 ? 16 : 0)) - m1;
                for (int l = 0; l < 32; ++l) *y++ = d2 * ((q[l] >> 4) + (x[b].qh[l] & u2 ? 16 : 0)) - m2;
            }
        }
    } break;
    case QREF_Q6_K: {                                   /* ggml-quants.c:1762-1791 */
        const blk_q6_K *x = (const blk_q6_K *)vx;
        for (int64_t b = 0; b < k / QKK; ++b) {
            const float d = H2F(x[b].d);
            for (int h = 0; h < 2; ++h, y += 128) {
                const uint8_t *ql = x[b].ql + 64 * h, *qh = x[b].qh + 32 * h;
                const int8_t *sc = x[b].scales + 8 * h;
                for (int l = 0; l < 32; ++l) {
                    const int g = l / 16;
                    const int8_t v0 = (int8_t)((ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                    const int8_t v1 = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                    const int8_t v2 = (int8_t)((ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                    const int8_t v3 = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                    y[l]      = d * sc[g + 0] * v0;
                    y[l + 32] = d * sc[g + 2] * v1;
                    y[l + 64] = d * sc[g + 4] * v2;
                    y[l + 96] = d * sc[g + 6] * v3;
                }
            }
        }
    } break;
    case QREF_Q8_K: {
        const blk_q8_K *x = (const blk_q8_K *)vx;
        for (int64_t b = 0; b < k / QKK; ++b)
            for (int j = 0; j < QKK; ++j) *y++ = x[b].d * x[b].qs[j];
    } break;
    default: abort();
    }
}

void qref_quantize_act(int type, const float *x, void *y, int64_t k, int flavour) {
    if (type == QREF_Q8_0) {
        if (flavour == QREF_ACT_X86) q8_0_from_f32_x86(x, (blk_q8_0 *)y, k / QK32);
        else                         q8_0_from_f32(x, (blk_q8_0 *)y, k / QK32);
    } else if (type == QREF_Q8_K) {
        q8_K_from_f32(x, (blk_q8_K *)y, k / QKK);
    } else if (type == QREF_Q8_1) {
        q8_1_from_f32(x, (blk_q8_1 *)y, k / QK32);
    } else {
        abort();
    }
}

/* ------------------------------------------------------------------------------------ */
/* generic vec_dots (ggml-cpu/quants.c) — float accumulation order preserved             */
/* ggml-cpu is built with the host ISA flags (GGML_NATIVE / -march), under which gcc's   */
/* default -ffp-contract=fast turns each `acc += a*b` accumulation into one FMA; the     */
/* explicit fmaf() calls below model exactly those contractions so the oracle reproduces */
/* ggml_vec_dot_*_generic bit-for-bit as upstream builds it.                             */
/* ------------------------------------------------------------------------------------ */
static float dot_q4_0(int n, const blk_q4_0 *x, const blk_q8_0 *y) {
    float acc = 0;
    for (int b = 0; b < n / QK32; ++b) {
        int s0 = 0, s1 = 0;
        for (int j = 0; j < 16; ++j) {
            s0 += ((x[b].qs[j] & 0x0F) - 8) * y[b].qs[j];
            s1 += ((x[b].qs[j] >> 4) - 8) * y[b].qs[j + 16];
        }
        acc = fmaf((float)(s0 + s1) * H2F(x[b].d), H2F(y[b].d), acc);
    }
    return acc;
}

static float dot_q8_0(int n, const blk_q8_0 *x, const blk_q8_0 *y) {
    float acc = 0;
    for (int b = 0; b < n / QK32; ++b) {
        int s = 0;
        for (int j = 0; j < QK32; ++j) s += x[b].qs[j] * y[b].qs[j];
        acc = fmaf((float)s, H2F(x[b].d) * H2F(y[b].d), acc);
    }
    return acc;
}

/* Q4_K/Q5_K share the 8-lane integer accumulation of quants.c:550-623 / 625-703:
 * lane l of aux32 collects sum over sub-blocks j of scale_j * q_w * q_x for positions
 * 8*i + l; the float reduction is sums[l] += d*aux32[l] per super-block, then
 * sumf -= dmin*sum(bsums*mins) per super-block, then sumf += sums[l] at the end. */
static float dot_k45(int n, const void *vx, const blk_q8_K *y, int has_hi) {
    const size_t stride = has_hi ? sizeof(blk_q5_K) : sizeof(blk_q4_K);
    float lanes[8] = {0};
    float acc = 0;
    for (int b = 0; b < n / QKK; ++b) {
        const uint8_t *blk = (const uint8_t *)vx + (size_t)b * stride;
        const uint16_t hd = (uint16_t)(blk[0] | (blk[1] << 8)), hdm = (uint16_t)(blk[2] | (blk[3] << 8));
        const uint8_t *sc12 = blk + 4;
        const uint8_t *qh = has_hi ? blk + 16 : NULL;
        const uint8_t *qs = has_hi ? blk + 48 : blk + 16;
        int8_t w[QKK];
        for (int c = 0; c < 4; ++c) {
            for (int l = 0; l < 32; ++l) {
                w[64 * c + l]      = (int8_t)(qs[32 * c + l] & 0xF);
                w[64 * c + 32 + l] = (int8_t)(qs[32 * c + l] >> 4);
                if (qh) {
                    w[64 * c + l]      += (qh[l] & (1u << (2 * c))) ? 16 : 0;
                    w[64 * c + 32 + l] += (qh[l] & (2u << (2 * c))) ? 16 : 0;
                }
            }
        }
        uint8_t s8[8], m8[8];
        for (int j = 0; j < 8; ++j) unpack_scale_min(sc12, j, &s8[j], &m8[j]);
        int msum = 0;
        for (int g = 0; g < 16; ++g) msum += y[b].bsums[g] * m8[g / 2];
        int32_t a32[8] = {0};
        for (int j = 0; j < 8; ++j)
            for (int i = 0; i < 32; ++i) a32[i % 8] += s8[j] * (int16_t)(y[b].qs[32 * j + i] * w[32 * j + i]);
        const float d = H2F(hd) * y[b].d;
        for (int l = 0; l < 8; ++l) lanes[l] = fmaf(d, (float)a32[l], lanes[l]);
        const float dmin = H2F(hdm) * y[b].d;
        acc = fmaf(-dmin, (float)msum, acc);
    }
    for (int l = 0; l < 8; ++l) acc += lanes[l];
    return acc;
}

static float dot_q6_K(int n, const blk_q6_K *x, const blk_q8_K *y) {
    float lanes[8] = {0};
    float acc = 0;
    for (int b = 0; b < n / QKK; ++b) {
        int8_t w[QKK];
        for (int h = 0; h < 2; ++h) {
            const uint8_t *ql = x[b].ql + 64 * h, *qh = x[b].qh + 32 * h;
            for (int l = 0; l < 32; ++l) {
                w[128 * h + l]      = (int8_t)((ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                w[128 * h + l + 32] = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                w[128 * h + l + 64] = (int8_t)((ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                w[128 * h + l + 96] = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
            }
        }
        int32_t a32[8] = {0};
        for (int g = 0; g < 16; ++g)
            for (int i = 0; i < 16; ++i) a32[i % 8] += x[b].scales[g] * (int16_t)(y[b].qs[16 * g + i] * w[16 * g + i]);
        const float d = H2F(x[b].d) * y[b].d;
        for (int l = 0; l < 8; ++l) lanes[l] = fmaf(d, (float)a32[l], lanes[l]);
    }
    for (int l = 0; l < 8; ++l) acc += lanes[l];
    return acc;
}

float qref_vec_dot(int type, int n, const void *x, const void *y) {
    switch (type) {
        case QREF_Q4_0: return dot_q4_0(n, (const blk_q4_0 *)x, (const blk_q8_0 *)y);
        case QREF_Q8_0: return dot_q8_0(n, (const blk_q8_0 *)x, (const blk_q8_0 *)y);
        case QREF_Q4_K: return dot_k45(n, x, (const blk_q8_K *)y, 0);
        case QREF_Q5_K: return dot_k45(n, x, (const blk_q8_K *)y, 1);
        case QREF_Q6_K: return dot_q6_K(n, (const blk_q6_K *)x, (const blk_q8_K *)y);
        case QREF_F32: {
            /* ggml_vec_dot_f32 reference semantics: plain f32 accumulation (double-free) */
            const float *a = (const float *)x, *b = (const float *)y;
            float s = 0;
            for (int i = 0; i < n; ++i) s += a[i] * b[i];
            return s;
        }
        default: abort();
    }
}

/* ------------------------------------------------------------------------------------ */
/* mul_mat / mul_mat_id                                                                  */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    const qref_tensor *src0, *src1, *ids;
    qref_tensor *dst;
    const uint8_t *act;      /* quantized src1, contiguous [ne13][ne12][ne11] rows */
    size_t act_row;
    int64_t n_jobs;
    int nth, ith;
} mm_job;

static void *mm_worker(void *arg) {
    mm_job *J = (mm_job *)arg;
    const qref_tensor *a = J->src0, *b = J->src1;
    qref_tensor *c = J->dst;
    const int64_t r2 = b->ne[2] / a->ne[2], r3 = b->ne[3] / a->ne[3];
    const int64_t ncols = b->ne[1] * b->ne[2] * b->ne[3];
    /* job = (column, block of 16 rows) — any partition gives identical results */
    const int64_t rblk = (a->ne[1] + 15) / 16;
    for (int64_t job = J->ith; job < ncols * rblk; job += J->nth) {
        const int64_t col = job / rblk, rb = job % rblk;
        const int64_t i13 = col / (b->ne[2] * b->ne[1]);
        const int64_t i12 = (col - i13 * b->ne[2] * b->ne[1]) / b->ne[1];
        const int64_t i11 = col - i13 * b->ne[2] * b->ne[1] - i12 * b->ne[1];
        const uint8_t *arow0 = (const uint8_t *)a->data + (i12 / r2) * a->nb[2] + (i13 / r3) * a->nb[3];
        const uint8_t *act = J->act + (size_t)col * J->act_row;
        float *out = (float *)((uint8_t *)c->data + i11 * c->nb[1] + i12 * c->nb[2] + i13 * c->nb[3]);
        for (int64_t r = rb * 16; r < IMIN(a->ne[1], rb * 16 + 16); ++r)
            out[r] = qref_vec_dot(a->type, (int)a->ne[0], arow0 + r * a->nb[1], act);
    }
    return NULL;
}

static int default_threads(int n) {
    if (n > 0) return n;
    long c = sysconf(_SC_NPROCESSORS_ONLN);
    return c > 0 ? (int)c : 1;
}

static void run_threads(mm_job *proto, int nth, void *(*fn)(void *)) {
    pthread_t *th = (pthread_t *)calloc((size_t)nth, sizeof(pthread_t));
    mm_job *jobs = (mm_job *)calloc((size_t)nth, sizeof(mm_job));
    for (int t = 0; t < nth; ++t) {
        jobs[t] = *proto;
        jobs[t].ith = t;
        jobs[t].nth = nth;
        if (t) pthread_create(&th[t], NULL, fn, &jobs[t]);
    }
    fn(&jobs[0]);
    for (int t = 1; t < nth; ++t) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
}

/* quantize every src1 row (ggml-cpu.c:1264-1299: row by row via the strides) */
static uint8_t *quantize_src1(const qref_tensor *src0, const qref_tensor *b, int flavour, size_t *row_bytes) {
    const int vt = qref_vec_dot_type(src0->type);
    const size_t rb = qref_row_size(vt, b->ne[0]);
    const int64_t nrow = b->ne[1] * b->ne[2] * b->ne[3];
    uint8_t *buf = (uint8_t *)malloc(rb * (size_t)(nrow ? nrow : 1));
    int64_t r = 0;
    for (int64_t i3 = 0; i3 < b->ne[3]; ++i3)
        for (int64_t i2 = 0; i2 < b->ne[2]; ++i2)
            for (int64_t i1 = 0; i1 < b->ne[1]; ++i1, ++r) {
                const float *x = (const float *)((const uint8_t *)b->data + i1 * b->nb[1] + i2 * b->nb[2] + i3 * b->nb[3]);
                if (vt == QREF_F32) memcpy(buf + r * rb, x, rb);
                else qref_quantize_act(vt, x, buf + r * rb, b->ne[0], flavour);
            }
    *row_bytes = rb;
    return buf;
}

int qref_mul_mat(const qref_tensor *src0, const qref_tensor *src1, qref_tensor *dst, int flavour, int n_threads) {
    if (src1->type != QREF_F32 || dst->type != QREF_F32) return -1;
    if (qref_vec_dot_type(src0->type) < 0) return -1;
    if (src0->ne[0] != src1->ne[0] || src1->ne[2] % src0->ne[2] || src1->ne[3] % src0->ne[3]) return -1;
    if (src0->nb[0] != qref_type_size(src0->type) || src1->nb[0] != 4 || dst->nb[0] != 4) return -1;
    mm_job J = {0};
    J.src0 = src0; J.src1 = src1; J.dst = dst;
    uint8_t *act = quantize_src1(src0, src1, flavour, &J.act_row);
    J.act = act;
    run_threads(&J, default_threads(n_threads), mm_worker);
    free(act);
    return 0;
}

/* mul_mat_id: row (e, t) of dst = as[ids[e,t]] @ b[:, e % b.ne1, t] (ggml.c:3043-3081,
 * ggml-cpu.c:1476-1655; grouping by expert does not change any single dot product) */
static void *mmid_worker(void *arg) {
    mm_job *J = (mm_job *)arg;
    const qref_tensor *as = J->src0, *b = J->src1, *ids = J->ids;
    qref_tensor *c = J->dst;
    const int64_t n_used = ids->ne[0], T = ids->ne[1];
    for (int64_t job = J->ith; job < n_used * T; job += J->nth) {
        const int64_t e = job % n_used, t = job / n_used;
        const int32_t ex = *(const int32_t *)((const uint8_t *)ids->data + e * ids->nb[0] + t * ids->nb[1]);
        const int64_t i11 = e % b->ne[1];
        const uint8_t *act = J->act + (size_t)(i11 + t * b->ne[1]) * J->act_row;
        const uint8_t *w = (const uint8_t *)as->data + ex * as->nb[2];
        float *out = (float *)((uint8_t *)c->data + e * c->nb[1] + t * c->nb[2]);
        for (int64_t r = 0; r < as->ne[1]; ++r) out[r] = qref_vec_dot(as->type, (int)as->ne[0], w + r * as->nb[1], act);
    }
    return NULL;
}

int qref_mul_mat_id(const qref_tensor *as, const qref_tensor *b, const qref_tensor *ids, qref_tensor *dst,
                    int flavour, int n_threads) {
    if (b->type != QREF_F32 || ids->type != QREF_I32 || qref_vec_dot_type(as->type) < 0) return -1;
    if (as->ne[0] != b->ne[0] || ids->ne[1] != b->ne[2] || ids->ne[0] % b->ne[1]) return -1;
    for (int64_t t = 0; t < ids->ne[1]; ++t)
        for (int64_t e = 0; e < ids->ne[0]; ++e) {
            const int32_t ex = *(const int32_t *)((const uint8_t *)ids->data + e * ids->nb[0] + t * ids->nb[1]);
            if (ex < 0 || ex >= as->ne[2]) return -2;
        }
    mm_job J = {0};
    J.src0 = as; J.src1 = b; J.ids = ids; J.dst = dst;
    uint8_t *act = quantize_src1(as, b, flavour, &J.act_row);
    J.act = act;
    run_threads(&J, default_threads(n_threads), mmid_worker);
    free(act);
    return 0;
}
