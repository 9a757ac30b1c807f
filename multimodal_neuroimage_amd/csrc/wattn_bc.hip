// Window attention for head_dim 2 on 6^3 windows, kind 0 (reference:
// WindowAttention_fusion.forward swinfusion_module.py:114-145 and Cross_WindowAttention.forward
// :213-246, and the autograd backward of both).  Head pairs are packed into f2 lanes of
// v_pk_fma_f32 (head 0, head 1), so a wave works on one head pair of one window at a time.
//
//   forward   wattn_fwd_bcs_kernel  lane = query pair (t, t + N/2); the wave walks the keys in
//                                   lock step, each key record an LDS broadcast read; online softmax;
//                                   a 4-wave workgroup streams the query pairs of a list of windows
//                                   (all lanes busy)
//   backward  wattn_bwd_q4k_kernel  lane = key quad (y + 3, z + 3 partners); the wave walks the
//                                   54 query quads; per step p and ds of 16 (query, key) pairs give
//                                   dk / dv (registers), the bias-table gradient (private LDS image)
//                                   and dq partials that a 64-lane butterfly reduces to the final
//                                   sums of the step's 4 queries -- one pass, no recomputation
//
// LDS facts that shape them (measured here, gfx950): a broadcast record is read 16 bytes at a time
// from a 16-byte-aligned address (ds_read_b128: 4 LDS cycles; the compiler's ds_read2_b64 pairs take
// 8; a misaligned b128 ran ~16x slower).  The window is a compile-time shape, so the key/query
// coordinates and codes are scalar loop counters, and every table access of a step is one address
// register plus immediate offsets.
//
// Bias-table gradient without atomics.  At one step the wave's lanes hold distinct keys against
// the same queries, so the relative-position entries they update, code(q) - code(k) + off, are
// pairwise distinct.  Each wave therefore read-modify-writes its OWN fp32 copy of the table in LDS
// with plain loads and stores: no atomics, no fixed-point scale, no max|dO| pre-pass (LDS float
// atomics measured ~8x slower).  A workgroup always serves the same head pair; its waves' copies
// are summed in a fixed order into one partial row per workgroup, and a fixed-order column sum
// (tokenops.hip) adds the rows: bitwise deterministic.
#include "wattn_common.h"

namespace mmni {

namespace bc {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// Broadcast records (every lane reads the same address) are read 16 bytes at a time from a
// 16-byte-aligned region: ds_read_b128 moves 16 B per lane in 4 LDS cycles, while the
// ds_read2_b64 the compiler forms from 8-byte reads takes 8 (MI355X_MICROARCH.md §LDS).  The
// region offsets below are rounded up to 16 B (a misaligned b128 measured ~16x slower).
__device__ __forceinline__ void ld_pair(const f2* p, f2& a, f2& b) {
    const f4 t = *reinterpret_cast<const f4*>(__builtin_assume_aligned(p, 16));
    a = (f2){t.x, t.y};
    b = (f2){t.z, t.w};
}
constexpr int align4(int n) { return (n + 3) & ~3; }   // floats, to a 16-byte boundary

__device__ __forceinline__ f2 splat(float x) { return (f2){x, x}; }
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 exp2_2(f2 x) { return (f2){fast_exp2(x.x), fast_exp2(x.y)}; }

// one head pair of a row in "pk" order: x[c] = (head 0 dim c, head 1 dim c); global rows hold
// (h0 c0, h0 c1, h1 c0, h1 c1)
struct Row {
    f2 x[2];
};

__device__ __forceinline__ Row load_row_pk(const float* src) {
    const float4 t = *reinterpret_cast<const float4*>(src);
    Row r;
    r.x[0] = (f2){t.x, t.z};
    r.x[1] = (f2){t.y, t.w};
    return r;
}

__device__ __forceinline__ void store_row_nat(float* dst, const Row& r, float scale) {
    *reinterpret_cast<float4*>(dst) =
        make_float4(r.x[0].x * scale, r.x[1].x * scale, r.x[0].y * scale, r.x[1].y * scale);
}

// Lane -> row-pair map of 6^3 windows.  A lane's table entries at one step are code(t) + const,
// and 8-byte LDS accesses conflict on (code mod 32) within 32-lane halves (ds_read_b64) and on
// (code mod 16) within 16-lane groups (ds_read2_b64, which the compiler forms from two steps).
// With code = 121 z + 11 y + x the identity order collides 2-way in every half; this order
// (a search over the 108 row pairs) leaves one 2-way collision in one group.
__constant__ unsigned char kPerm666[108] = {7, 12, 16, 26, 30, 32, 38, 40, 48, 63, 81, 82, 83, 91, 92, 101, 4, 29, 35, 43, 44, 51, 65, 66, 69, 77, 79, 85, 87, 89, 95, 97, 0, 1, 5, 6, 9, 10, 15, 31, 53, 56, 61, 62, 68, 78, 90, 103, 3, 13, 21, 33, 34, 46, 49, 58, 59, 67, 75, 88, 93, 100, 102, 106, 8, 14, 17, 18, 22, 28, 39, 41, 42, 45, 47, 52, 72, 76, 80, 86, 2, 20, 23, 24, 27, 36, 50, 54, 57, 71, 74, 84, 94, 98, 104, 107, 11, 19, 25, 37, 55, 60, 64, 70, 73, 96, 99, 105};

// compile-time window (WD even): tokens t = (i*WH + j)*WW + k, relative codes
// code = i*TW + j*TH + k, table rows TSZ, the second half starts DC codes later
template <int WD, int WH, int WW>
struct Win {
    static constexpr int N = WD * WH * WW, H = N / 2;
    static constexpr int TH = 2 * WW - 1, TW = (2 * WH - 1) * TH, TSZ = (2 * WD - 1) * TW;
    static constexpr int OFF = (WD - 1) * TW + (WH - 1) * TH + (WW - 1);
    static constexpr int DC = (WD / 2) * TW;
    static_assert(WD % 2 == 0, "pairing needs whole planes");
    static_assert(WD == 6 && WH == 6 && WW == 6, "lane order kPerm666 is for 6^3 windows");
};

// Per-window shift-region state.  A window spans several regions only if it is the last one
// along a shifted axis (shift_region); then the region of local coordinate c on that axis is
// 1 + (c >= w - s).  The region code packs one split bit per axis.
struct Regions {
    bool masked;
    int lz, ly, lx;   // split points (local coordinate), or a value beyond the window (no split)
};

__device__ __forceinline__ Regions window_regions(const WGeom& g, int w) {
    const int wx = w % g.nWw;
    w /= g.nWw;
    const int wy = w % g.nWh;
    w /= g.nWh;
    const int wz = w % g.nWd;
    Regions r;
    const bool mz = g.sd && wz == g.nWd - 1, my = g.sh && wy == g.nWh - 1, mx = g.sw && wx == g.nWw - 1;
    r.masked = mz || my || mx;
    r.lz = mz ? g.wd - g.sd : 1 << 20;
    r.ly = my ? g.wh - g.sh : 1 << 20;
    r.lx = mx ? g.ww - g.sw : 1 << 20;
    return r;
}

__device__ __forceinline__ int region_code(const Regions& r, int i, int j, int k) {
    return ((i >= r.lz) << 2) | ((j >= r.ly) << 1) | (k >= r.lx);
}

// The backward may fold p = 2^(s - lse) into 2^s * 2^-lse, with 2^-lse multiplied into dO and
// -delta once per row, when |lse| (log2 domain) <= kFoldMax for the rows involved: then 2^s <=
// 2^kFoldMax and 2^-lse >= 2^-kFoldMax, so neither factor over- or underflows where p matters and
// the per-score subtract disappears.  Rows outside the bound take the subtracting loop.
constexpr float kFoldMax = 30.0f;

__device__ __forceinline__ bool fold_ok(f2 l) { return fabsf(l.x) <= kFoldMax && fabsf(l.y) <= kFoldMax; }

}  // namespace bc

using bc::f2;
using bc::Row;

// ------------------------------------------------------------------------------------
// forward: lane = query pair (t, t + H); keys (n, n + H) broadcast from LDS as in pass A.
// Online softmax with a lazy reference: scores are taken relative to a per-row reference m
// (initialised from the first key) and m is raised -- with the rescale of l and o -- only when a
// score exceeds it by more than kLazy (wave-uniform test).  So p = exp2(s - m) <= 2^kLazy, no
// overflow, and the common step costs one exp per score and no rescale.  No software prefetch
// of the next key: the 105-VGPR loop runs 4 waves per SIMD (the LDS footprint allows 8 blocks
// per CU), and the other waves hide the broadcast reads.
// ------------------------------------------------------------------------------------
constexpr float kLazy = 8.0f;
// Bounded rows skip the reference altogether: when |s| <= |q| max|k| + max|bias| <= kFwdBound for
// every key of a row (Cauchy-Schwarz on the log2-scaled scores), p = 2^s lies in
// [2^-kFwdBound, 2^kFwdBound] (masked keys: ~2^-144, i.e. 0) and l, o stay far inside fp32, so the
// common step is the bare score, one exp, l += p and o += p v.
constexpr float kFwdBound = 30.0f;

template <int WD, int WH, int WW, bool MASKED, bool BOUNDED>
__device__ __forceinline__ void fwd_loop(const Row (&q)[2], f2 (&m)[2], f2 (&l)[2], Row (&o)[2], int cq,
                                         const int (&rq)[2], const bc::Regions& reg, const float* tab,
                                         const float* kv_s) {
    using Wn = bc::Win<WD, WH, WW>;
    constexpr int EB = 8;
    const char* tb = reinterpret_cast<const char*>(tab);
    const uint32_t lane_base = (uint32_t)((cq - Wn::DC) * EB);
    const f2* kv2 = reinterpret_cast<const f2*>(kv_s);
    f2 kk[2][2], vv[2][2], tbm, tb0, tbp;
    auto fetch = [&](const f2* kvk, const char* pe, f2 (&k_)[2][2], f2 (&v_)[2][2], f2& m_, f2& z_, f2& p_) {
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            bc::ld_pair(kvk + v * 4, k_[v][0], k_[v][1]);
            bc::ld_pair(kvk + v * 4 + 2, v_[v][0], v_[v][1]);
        }
        m_ = *reinterpret_cast<const f2*>(pe);
        z_ = *reinterpret_cast<const f2*>(pe + Wn::DC * EB);
        p_ = *reinterpret_cast<const f2*>(pe + 2 * Wn::DC * EB);
    };
    fetch(kv2, tb + lane_base, kk, vv, tbm, tb0, tbp);
    if (BOUNDED) {
        m[0] = m[1] = bc::splat(0.f);
    } else {   // the reference: each row's exact maximum over the first key's two rows
        int rk[2] = {0, 0};
        if (MASKED) {
            rk[0] = bc::region_code(reg, 0, 0, 0);
            rk[1] = bc::region_code(reg, WD / 2, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            f2 sv[2];
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                f2 base = (u == v) ? tb0 : (u == 0 ? tbm : tbp);
                if (MASKED) base += bc::splat(rk[v] == rq[u] ? 0.f : kMask2);
                f2 s = bc::pfma(q[u].x[0], kk[v][0], base);
                sv[v] = bc::pfma(q[u].x[1], kk[v][1], s);
            }
            m[u] = (f2){fmaxf(sv[0].x, sv[1].x), fmaxf(sv[0].y, sv[1].y)};
        }
    }
    for (int i = 0; i < WD / 2; ++i) {
        for (int j = 0; j < WH; ++j) {
            const int code0 = i * Wn::TW + j * Wn::TH;
            const f2* kvr = kv2 + (i * WH + j) * WW * 8;
            const char* trow = tb + (lane_base - (uint32_t)((code0 + WW - 1) * EB));
#pragma unroll
            for (int k = 0; k < WW; ++k) {
                fetch(kvr + k * 8, trow + (WW - 1 - k) * EB, kk, vv, tbm, tb0, tbp);
                int rk[2] = {0, 0};
                if (MASKED) {
                    rk[0] = bc::region_code(reg, i, j, k);
                    rk[1] = bc::region_code(reg, i + WD / 2, j, k);
                }
                f2 s[2][2];
                float smax = -INFINITY;
#pragma unroll
                for (int u = 0; u < 2; ++u) {
#pragma unroll
                    for (int v = 0; v < 2; ++v) {
                        const f2 t = (u == v) ? tb0 : (u == 0 ? tbm : tbp);
                        f2 base = BOUNDED ? t : t - m[u];
                        if (MASKED) base += bc::splat(rk[v] == rq[u] ? 0.f : kMask2);
                        f2 sv = bc::pfma(q[u].x[0], kk[v][0], base);
                        sv = bc::pfma(q[u].x[1], kk[v][1], sv);
                        s[u][v] = sv;
                        if (!BOUNDED) smax = fmaxf(smax, fmaxf(sv.x, sv.y));
                    }
                }
                if (!BOUNDED && __any(smax > kLazy)) {   // rare: raise the reference of the rows that need it
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const f2 up = (f2){fmaxf(fmaxf(s[u][0].x, s[u][1].x), 0.f),
                                           fmaxf(fmaxf(s[u][0].y, s[u][1].y), 0.f)};
                        const f2 alpha = bc::exp2_2(-up);
                        l[u] *= alpha;
                        o[u].x[0] *= alpha;
                        o[u].x[1] *= alpha;
                        m[u] += up;
                        s[u][0] -= up;
                        s[u][1] -= up;
                    }
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
#pragma unroll
                    for (int v = 0; v < 2; ++v) {
                        const f2 p = bc::exp2_2(s[u][v]);
                        l[u] += p;
                        o[u].x[0] = bc::pfma(p, vv[v][0], o[u].x[0]);
                        o[u].x[1] = bc::pfma(p, vv[v][1], o[u].x[1]);
                    }
                }
                // the bounded step has no branch: keep the compiler from hoisting the whole row's
                // broadcast reads (they spill at the 4-wave register budget)
                if (BOUNDED) __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// "quad" layout of 6^3 windows: the row quad {b, b + 18, b + 108, b + 126} (the (y + 3, z + 3)
// partners of b = (z', y', x), z', y' < 3): 54 quads per window, one lane each, one wave per (window,
// head pair).  The wave walks the other side's 54 quads in lock step, so each broadcast record feeds
// 16 (query, key) pairs instead of 4, and the 16 pairs of a step touch only 9 table entries
// (relative offsets a * 3 TW + b * 3 TH, a, b in {-1, 0, 1}).  The bases' codes hit each of the 32
// 8-byte bank pairs once in lanes 0-31 and at most once in lanes 32-53 (kPermQ), so every
// per-lane table access is conflict-free.  The 9 x 54 entries of one step are pairwise distinct
// (codes of bases differ by less than 3 in every digit, the slot offsets by multiples of 3), so the
// private table read-modify-write of a step never aliases across lanes.
// ------------------------------------------------------------------------------------
namespace q4 {
constexpr int NB = 54;                              // row quads per window
constexpr int TW = 121, TH = 11, OFF = 665, TSZ = 1331;
constexpr int EB = 8;                               // table entry: f2 over the head pair
constexpr int WAVES = 4;                            // waves per workgroup (one head pair per workgroup)
__constant__ unsigned char kPermQ[NB] = {0,  1,  2,  3,  4,  5,  26, 27, 28, 29, 50, 6,  7,  8,  9,  10, 11, 32,
                                         33, 34, 35, 39, 12, 13, 14, 15, 16, 17, 21, 22, 23, 44, 18, 19, 20, 24,
                                         25, 30, 31, 36, 37, 38, 40, 41, 42, 43, 45, 46, 47, 48, 49, 51, 52, 53};
__device__ __forceinline__ int base_token(int b) { return (b / 18) * 36 + ((b / 6) % 3) * 6 + b % 6; }
__device__ __forceinline__ int base_code(int b) { return (b / 18) * TW + ((b / 6) % 3) * TH + b % 6; }
// combo (u, v) of query row u and key row v (bit 0: +3 y, bit 1: +3 z) -> table entry slot e and
// its code offset D
constexpr int slot(int u, int v) { return ((u >> 1) - (v >> 1) + 1) * 3 + ((u & 1) - (v & 1) + 1); }
constexpr int dcode(int e) { return (e / 3 - 1) * 3 * TW + (e % 3 - 1) * 3 * TH; }

// work of one wave: windows w = xcd + 8 j of its head pair (the head-pair workgroups of a window
// share an XCD's L2)
struct Work {
    int hp, j0, dj, xcd;
};
__device__ __forceinline__ Work work(int NHG, int wave) {
    Work k;
    k.xcd = blockIdx.x & 7;
    const int slot = blockIdx.x >> 3, nslots = gridDim.x >> 3;
    k.hp = slot % NHG;
    const int nblk = (nslots - k.hp + NHG - 1) / NHG;
    k.j0 = (slot / NHG) * WAVES + wave;
    k.dj = nblk * WAVES;
    return k;
}
}  // namespace q4

// 64-lane butterfly helpers of the merged backward's reductions: v_permlane32_swap /
// v_permlane16_swap exchange register halves across lane halves (one instruction per register
// pair), DPP forms x + partner(x) within a row (scripts/check_permlane.hip checks the semantics).
namespace q4 {
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ void swap32(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap16(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
}  // namespace q4

// ------------------------------------------------------------------------------------
// key-stationary merged backward (the C3 kernel).  A lane owns the KEY quad {b, b + 18, b + 108,
// b + 126} (k, v and the dk, dv accumulators stay in its registers for the whole window) and the
// wave walks the 54 QUERY quads, each a broadcast record of 4 rows x (q * scale * log2 e, dO) plus
// -delta and lse.  Per step a lane forms p and ds of its 16 (query, key) pairs once; dk and dv
// accumulate in place, and only dq -- 4 rows x 2 dims x 2 heads = 16 floats -- needs the 64-lane
// sum (reduce16), whose results replace the step's dead record.  (The query-stationary walk of
// r2g-r3f held dq in registers and reduced the step's 32 dk / dv values instead: 24 lane-swap
// instructions per step against 12 here, 343 instructions per step against 308.)  The bias-table
// entries of a step are code(q) - code(k) + off with the lane's key code negated: kPermQ still
// spreads them over the 32 bank pairs, and they stay pairwise distinct, so the private table
// image is still updated with plain loads and stores.
//
// LDS: the query records (192 B per quad) do not fit next to four table images for the whole
// window, so each wave walks the window in two halves -- quad rows 0-4 (30 quads) and 5-8 (24) --
// through one 30-record ring: the owners of a half's quads stage its records, the wave walks it,
// the owners write their dq rows out of the ring, and the next half is staged in its place.  The
// fold of 2^-lse into dO and -delta is decided per half.  (Measured and dropped: loading the
// second half's rows by LDS-DMA into the dead slots during the first half's last row; the spills
// it forced cost more than the hidden latency, r3m: 2.73 against 2.52 ms.)
// ------------------------------------------------------------------------------------
namespace k4 {
constexpr int REC = 192;                            // q~ f4 + dO f4 per row (128 B) | -delta f2 x 4 | lse2 f2 x 4
constexpr int HALF_ROWS = 5;                        // quad rows (6 quads each) of the first half
constexpr int RING = HALF_ROWS * 6 * REC;           // 5760 B per wave
constexpr int WAVES = 4;
constexpr int TABB = q4::TSZ * q4::EB;              // 10648 B per table image
constexpr int TAB = WAVES * RING;                   // bias table after the rings
constexpr int DT = (TAB + TABB + 15) & ~15;         // gradient images, one per wave
constexpr int LDS = DT + WAVES * TABB;              // 76288 B: two workgroups per CU
constexpr int DMN = 3 * q4::TW + 3 * q4::TH;        // 396: slot offsets dcode(e) + DMN >= 0
static_assert(q4::OFF - (2 * q4::TW + 2 * q4::TH + 5) - DMN >= 0, "lane table bases must be >= 0");

// 8 f2 dq partials per lane, value i = (u, c, h) in P[u * 2 + c].{x: h0, y: h1} -> lane l returns
// the 64-lane sum of value (u = l >> 4 & 3, c = l >> 3 & 1, h = l >> 2 & 1).  Stages 1-2 swap
// register halves across lane halves; stages 3-4 form BOTH candidate sums x + dpp(x) and keep the
// one the lane bit selects; 5-6 add the quad partners.  Fixed lane tree: bitwise deterministic.
__device__ __forceinline__ float reduce16(f2 (&P)[8], int lane) {
    f2 R[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {   // lanes 0-31 keep rows u = 0, 1; lanes 32-63 rows 2, 3
        float a0 = P[k].x, b0 = P[k + 4].x, a1 = P[k].y, b1 = P[k + 4].y;
        q4::swap32(a0, b0);
        q4::swap32(a1, b1);
        R[k] = (f2){a0, a1} + (f2){b0, b1};
    }
    f2 S[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {   // rows 0, 2 of 16 lanes keep u & 1 = 0, rows 1, 3 keep u & 1 = 1
        float a0 = R[k].x, b0 = R[k + 2].x, a1 = R[k].y, b1 = R[k + 2].y;
        q4::swap16(a0, b0);
        q4::swap16(a1, b1);
        S[k] = (f2){a0, a1} + (f2){b0, b1};
    }
    const bool b3 = lane & 8, b2 = lane & 4;
    // lane bit 3: dim c (row_ror:8 partner = lane ^ 8)
    const float lo_x = S[0].x + q4::dpp<0x128>(S[0].x), hi_x = S[1].x + q4::dpp<0x128>(S[1].x);
    const float lo_y = S[0].y + q4::dpp<0x128>(S[0].y), hi_y = S[1].y + q4::dpp<0x128>(S[1].y);
    const float Tx = b3 ? hi_x : lo_x, Ty = b3 ? hi_y : lo_y;
    // lane bit 2: head h (row_half_mirror partner = lane ^ 7 within 8), then quad xor 2 and xor 1
    const float ux = Tx + q4::dpp<0x141>(Tx), uy = Ty + q4::dpp<0x141>(Ty);
    const float U = b2 ? uy : ux;
    const float V = U + q4::dpp<0x4E>(U);
    return V + q4::dpp<0xB1>(V);
}
}  // namespace k4

// walk of the query-quad rows [r0, r1), whose records start at ring offset recw (row r0)
template <bool MASKED, bool FOLD>
__device__ __forceinline__ void q4k_walk(int r0, int r1, const Row (&kk)[4], const Row (&vv)[4], Row (&dk)[4],
                                         Row (&dv)[4], const int (&rk)[4], const bc::Regions& reg, char* sm,
                                         int recw, int dtw, uint32_t lane_e, f2 live) {
    using namespace q4;
    const int lane = threadIdx.x & 63;
    // where this lane's dq sum (u, c, h) goes in the step's dead record: [u][h c], the row order
    const int soff = ((lane >> 4) & 3) * 16 + ((lane >> 2) & 1) * 8 + ((lane >> 3) & 1) * 4;
    // The table image offset goes through an empty asm after each step's stores, so the compiler
    // treats the next step's table reads as possibly aliasing them (other lanes' entries) and keeps
    // them behind the stores; LDS executes a wave's accesses in order, so no wait is needed.
    int dto = dtw;   // this wave's table-gradient image (an LDS offset: the accesses stay ds_*)
    for (int r = r0; r < r1; ++r) {
        const int zr = r / 3, yr = r - 3 * (r / 3);
        const uint32_t trow = lane_e + (uint32_t)((zr * TW + yr * TH) * EB);
        char* rrow = sm + recw + (r - r0) * 6 * k4::REC;
#pragma unroll
        for (int x = 0; x < 6; ++x) {
            f2 P[8];
            __builtin_amdgcn_sched_barrier(0);
            {
                char* dp = sm + dto + trow;
                const char* tp = sm + k4::TAB + trow;
                const char* rec = rrow + x * k4::REC;
                f2 od[9], bt[9];
#pragma unroll
                for (int e = 0; e < 9; ++e) od[e] = *reinterpret_cast<const f2*>(dp + (x + dcode(e) + k4::DMN) * EB);
                Row qs[4], dO[4];
                f2 nd[4], ls[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    bc::ld_pair(reinterpret_cast<const f2*>(rec + u * 32), qs[u].x[0], qs[u].x[1]);
                    bc::ld_pair(reinterpret_cast<const f2*>(rec + u * 32 + 16), dO[u].x[0], dO[u].x[1]);
                }
                bc::ld_pair(reinterpret_cast<const f2*>(rec + 128), nd[0], nd[1]);
                bc::ld_pair(reinterpret_cast<const f2*>(rec + 144), nd[2], nd[3]);
#pragma unroll
                for (int u = 0; u < 4; ++u) nd[u] *= live;   // spare lanes: ds = p * 0 = 0
                if (!FOLD) {
                    bc::ld_pair(reinterpret_cast<const f2*>(rec + 160), ls[0], ls[1]);
                    bc::ld_pair(reinterpret_cast<const f2*>(rec + 176), ls[2], ls[3]);
                }
#pragma unroll
                for (int e = 0; e < 9; ++e) bt[e] = *reinterpret_cast<const f2*>(tp + (x + dcode(e) + k4::DMN) * EB);
                int rq[4] = {0, 0, 0, 0};
                if (MASKED) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) rq[u] = bc::region_code(reg, zr + 3 * (u >> 1), yr + 3 * (u & 1), x);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        const int e = slot(u, v);
                        f2 base = FOLD ? bt[e] : bt[e] - ls[u];
                        if (MASKED) base += bc::splat(rk[v] == rq[u] ? 0.f : kMask2);
                        f2 s = bc::pfma(qs[u].x[0], kk[v].x[0], base);
                        s = bc::pfma(qs[u].x[1], kk[v].x[1], s);
                        const f2 p = bc::exp2_2(s);
                        f2 tt = bc::pfma(dO[u].x[0], vv[v].x[0], nd[u]);
                        tt = bc::pfma(dO[u].x[1], vv[v].x[1], tt);
                        const f2 ds = p * tt;
                        if (v == 0) {   // first key: plain products (P is zero)
                            P[u * 2] = ds * kk[0].x[0];
                            P[u * 2 + 1] = ds * kk[0].x[1];
                        } else {
                            P[u * 2] = bc::pfma(ds, kk[v].x[0], P[u * 2]);
                            P[u * 2 + 1] = bc::pfma(ds, kk[v].x[1], P[u * 2 + 1]);
                        }
                        dk[v].x[0] = bc::pfma(ds, qs[u].x[0], dk[v].x[0]);
                        dk[v].x[1] = bc::pfma(ds, qs[u].x[1], dk[v].x[1]);
                        dv[v].x[0] = bc::pfma(p, dO[u].x[0], dv[v].x[0]);
                        dv[v].x[1] = bc::pfma(p, dO[u].x[1], dv[v].x[1]);
                        od[e] += ds;
                    }
                    // pin the accumulators here: without it the compiler defers the dk / dv
                    // updates past the step (holding every p and ds: spilled)
#pragma unroll
                    for (int v = 0; v < 4; ++v)
                        asm volatile("" : "+v"(dk[v].x[0]), "+v"(dk[v].x[1]), "+v"(dv[v].x[0]), "+v"(dv[v].x[1]));
                }
#pragma unroll
                for (int e = 0; e < 9; ++e) *reinterpret_cast<f2*>(dp + (x + dcode(e) + k4::DMN) * EB) = od[e];
            }
            asm volatile("" : "+v"(dto));   // next reads: behind the stores above (see dto)
            const float sum = k4::reduce16(P, lane);
            // the final dq sums of query quad (r, x) replace its record (read above: LDS runs a
            // wave's accesses in order); the owner lane writes the rows out after the half
            if ((lane & 3) == 0) *reinterpret_cast<float*>(rrow + x * k4::REC + soff) = sum;
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// stage the query records of a half into the wave's ring; returns the fold flag of the half (every
// row of the half has |lse| <= kFoldMax in the log2 domain)
__device__ __forceinline__ bool q4k_stage(const WAArgs& a, bool mine, int slot_off, const int64_t (&row)[4], int coff,
                                          int hp, int NHT, f2 qscale) {
    Row qs[4], dO[4];
    f2 nd[4], ls[4];
    bool ok = true;
    if (mine) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            // opaque row copies: otherwise the compiler forms every row's q / dO / o / lse / dq
            // address once per window, keeps them across both walks and spills them (reloaded here
            // at memory latency)
            int64_t rw = row[u];
            asm volatile("" : "+v"(rw));
            qs[u] = bc::load_row_pk(a.q + rw * a.qs + coff);
            dO[u] = bc::load_row_pk(a.dout + rw * a.os + coff);
            const Row o = bc::load_row_pk(a.o + rw * a.os + coff);
            qs[u].x[0] *= qscale;
            qs[u].x[1] *= qscale;
            nd[u] = -bc::pfma(o.x[0], dO[u].x[0], o.x[1] * dO[u].x[1]);
            ls[u] = (f2){a.lse[rw * NHT + 2 * hp], a.lse[rw * NHT + 2 * hp + 1]} * kLog2e;
            ok = ok && bc::fold_ok(ls[u]);
        }
    }
    const bool fold = __all(ok);   // lanes outside the half vote true
    if (mine) {
        extern __shared__ __attribute__((aligned(16))) float smem[];
        char* rec = reinterpret_cast<char*>(smem) + slot_off;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (fold) {
                const f2 e = bc::exp2_2(-ls[u]);
                dO[u].x[0] *= e;
                dO[u].x[1] *= e;
                nd[u] *= e;
            }
            *reinterpret_cast<bc::f4*>(rec + u * 32) = (bc::f4){qs[u].x[0].x, qs[u].x[0].y, qs[u].x[1].x, qs[u].x[1].y};
            *reinterpret_cast<bc::f4*>(rec + u * 32 + 16) =
                (bc::f4){dO[u].x[0].x, dO[u].x[0].y, dO[u].x[1].x, dO[u].x[1].y};
        }
        *reinterpret_cast<bc::f4*>(rec + 128) = (bc::f4){nd[0].x, nd[0].y, nd[1].x, nd[1].y};
        *reinterpret_cast<bc::f4*>(rec + 144) = (bc::f4){nd[2].x, nd[2].y, nd[3].x, nd[3].y};
        *reinterpret_cast<bc::f4*>(rec + 160) = (bc::f4){ls[0].x, ls[0].y, ls[1].x, ls[1].y};
        *reinterpret_cast<bc::f4*>(rec + 176) = (bc::f4){ls[2].x, ls[2].y, ls[3].x, ls[3].y};
    }
    asm volatile("" ::: "memory");   // the records are written before the walk reads them
    return fold;
}

// dq rows of a half's quads from their ring slots (the walk left the sums there)
__device__ __forceinline__ void q4k_flush(const WAArgs& a, bool mine, const char* rec, const int64_t (&row)[4],
                                          int coff) {
    if (mine) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            int64_t rw = row[u];
            asm volatile("" : "+v"(rw));   // as in q4k_stage
            const bc::f4 d = *reinterpret_cast<const bc::f4*>(rec + u * 16);
            *reinterpret_cast<bc::f4*>(a.dq + rw * a.qs + coff) = d * a.scale;
        }
    }
    asm volatile("" ::: "memory");   // the next half's records stay behind these reads
}

__global__ __launch_bounds__(k4::WAVES * 64) __attribute__((amdgpu_waves_per_eu(2)))
void wattn_bwd_q4k_kernel(WAArgs a, float* part) {
    using namespace q4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    char* sm = reinterpret_cast<char*>(smem);
    const WGeom& g = a.g;
    const int NHG = a.hsplit, NHT = 2 * NHG;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = tid >> 6;
    const Work wk = work(NHG, wave);
    float* tab = reinterpret_cast<float*>(sm + k4::TAB);
    for (int e = tid; e < TSZ * 2; e += blockDim.x) tab[e] = a.table[(e >> 1) * NHT + 2 * wk.hp + (e & 1)] * kLog2e;
    float* dtf = reinterpret_cast<float*>(sm + k4::DT);
    for (int e = tid; e < k4::WAVES * TSZ * 2; e += blockDim.x) dtf[e] = 0.f;
    __syncthreads();
    // Spare lanes (54..63) run every step with k = v = 0 and -delta masked to 0, so their ds and dq
    // partials are exact zeros and their table-image updates add zero.  They share the virtual key
    // code kSpareCode: its entries code(q) - kSpareCode + off + dcode(e) never meet a real lane's at
    // the same step (kSpareCode - code(b) + dcode(e) - dcode(e') has a units digit 10 - x of 5..10,
    // never a multiple of 11, while the slot offsets are) and stay inside the image (259..1320).
    constexpr int kSpareCode = 10;
    const bool lane_ok = lane < NB;
    const int beta = lane_ok ? (int)kPermQ[lane] : 0;
    const int tb0 = base_token(beta);
    const int bz = beta / 18, by = (beta / 6) % 3, bx = beta % 6, brow = beta / 6;
    const uint32_t lane_e = (uint32_t)((OFF - (lane_ok ? base_code(beta) : kSpareCode) - k4::DMN) * EB);
    const f2 live = bc::splat(lane_ok ? 1.f : 0.f);
    const int recw = wave * k4::RING, dtw = k4::DT + wave * k4::TABB;
    const int coff = wk.hp * 4;
    const f2 qscale = bc::splat(a.scale * kLog2e);
    for (int j = wk.j0;; j += wk.dj) {
        const int w = wk.xcd + 8 * j;
        if (w >= g.nwin) break;
        const bc::Regions reg = bc::window_regions(g, w);
        Row kk[4], vv[4], dk[4], dv[4];
        int rk[4] = {0, 0, 0, 0};
        int64_t row[4] = {0, 0, 0, 0};
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            kk[v].x[0] = kk[v].x[1] = vv[v].x[0] = vv[v].x[1] = bc::splat(0.f);
            dk[v].x[0] = dk[v].x[1] = dv[v].x[0] = dv[v].x[1] = bc::splat(0.f);
        }
        int tb = tb0;
        asm volatile("" : "+v"(tb));   // recompute the lane's token coordinates per window (hoisted, they spill)
        if (lane_ok) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const TokenInfo ti = token_info(g, w, tb + (v & 1) * 18 + (v >> 1) * 108);
                row[v] = ti.row;
                rk[v] = bc::region_code(reg, bz + 3 * (v >> 1), by + 3 * (v & 1), bx);
                kk[v] = bc::load_row_pk(a.k + ti.row * a.ks + coff);
                vv[v] = bc::load_row_pk(a.v + ti.row * a.vs + coff);
            }
        }
        // half A: quad rows 0-4 (ring slots 0-29), half B: rows 5-8 (slots 0-23)
#define MMNI_Q4K(M, F, R0, R1, RB) q4k_walk<M, F>(R0, R1, kk, vv, dk, dv, rk, reg, sm, RB, dtw, lane_e, live)
#define MMNI_WALK(R0, R1, RB)                                                       \
    do {                                                                        \
        if (fold) {                                                             \
            if (reg.masked) MMNI_Q4K(true, true, R0, R1, RB);                   \
            else MMNI_Q4K(false, true, R0, R1, RB);                             \
        } else {                                                                \
            if (reg.masked) MMNI_Q4K(true, false, R0, R1, RB);                  \
            else MMNI_Q4K(false, false, R0, R1, RB);                            \
        }                                                                       \
    } while (0)
        for (int half = 0; half < 2; ++half) {
            const int r0 = half ? k4::HALF_ROWS : 0, r1 = half ? 9 : k4::HALF_ROWS;
            const bool mine = lane_ok && brow >= r0 && brow < r1;
            const int slot_off = recw + (beta - 6 * r0) * k4::REC;
            const bool fold = q4k_stage(a, mine, slot_off, row, coff, wk.hp, NHT, qscale);
            MMNI_WALK(r0, r1, recw);
            q4k_flush(a, mine, sm + slot_off, row, coff);
        }
#undef MMNI_WALK
#undef MMNI_Q4K
        if (lane_ok) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                bc::store_row_nat(a.dk + row[v] * a.ks + coff, dk[v], kLn2);   // q carried scale * log2 e
                bc::store_row_nat(a.dv + row[v] * a.vs + coff, dv[v], 1.0f);
            }
        }
    }
    __syncthreads();
    float* prow = part + (int64_t)blockIdx.x * TSZ * NHT;
    for (int e = tid; e < TSZ * NHT; e += blockDim.x) {
        const int r = e / NHT, c = e - r * NHT;
        float v = 0.f;
        if ((c >> 1) == wk.hp) {
            const int o = r * 2 + (c & 1);
            v = ((dtf[o] + dtf[TSZ * 2 + o]) + dtf[TSZ * 4 + o]) + dtf[TSZ * 6 + o];
        }
        prow[e] = v;
    }
}

// ------------------------------------------------------------------------------------
// forward with streaming lanes.  A (window, head pair) has 108 query pairs, so the two-wave
// workgroup above leaves 20 of its 128 lanes idle (84% lane use).  Here a 4-wave workgroup owns a
// list of windows of one head pair and walks their query pairs as one sequence of slots, 256 per
// round: every lane works, and a wave spans at most two windows (two broadcast addresses per
// record read, their ring slots 16 bytes apart in bank order).  Each window's key records are
// staged once into a 4-slot ring (a round touches at most 4 windows), with its max |k|^2 for the
// bounded-step test.
// ------------------------------------------------------------------------------------
namespace fs {
constexpr int WAVES = 4, RING = 4;
constexpr int REC = 108 * 64;          // records of one window (pair t: keys t, t + 108)
constexpr int SLOT = REC + 16;         // ring stride: consecutive slots 16 B apart modulo 128 B
}  // namespace fs

template <int WD, int WH, int WW>
__global__ __launch_bounds__(fs::WAVES * 64) __attribute__((amdgpu_waves_per_eu(4)))
void wattn_fwd_bcs_kernel(WAArgs a) {
    using Wn = bc::Win<WD, WH, WW>;
    constexpr int H = Wn::H, TSZ = Wn::TSZ;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int NHG = a.hsplit, NHT = 2 * NHG;
    float* tab_s = smem;                                        // [TSZ] f2: bias * log2e
    char* ring = reinterpret_cast<char*>(tab_s + bc::align4(TSZ * 2));
    float* red = reinterpret_cast<float*>(ring + fs::RING * fs::SLOT);   // [WAVES][2] max|bias|; [RING][2][2] max|k|^2
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    // workgroup -> (XCD, head pair, window list): windows w = xcd + 8 (j0 + i), i < cnt
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslots = gridDim.x >> 3;
    const int hp = slot % NHG, kb = slot / NHG, nblk = (nslots - hp + NHG - 1) / NHG;
    const int nj = (g.nwin - xcd + 7) / 8, per = (nj + nblk - 1) / nblk, j0 = kb * per;
    const int cnt = nj - j0 < 0 ? 0 : (nj - j0 < per ? nj - j0 : per);
    float tabs = 0.f;
    for (int e = tid; e < TSZ * 2; e += blockDim.x) {
        const float x = a.table[(e >> 1) * NHT + 2 * hp + (e & 1)] * kLog2e;
        tab_s[e] = x;
        tabs = fmaxf(tabs, fabsf(x));
    }
    for (int off = 2; off < 64; off <<= 1) tabs = fmaxf(tabs, __shfl_xor(tabs, off));
    if (lane < 2) red[wave * 2 + lane] = tabs;
    __syncthreads();
    f2 tmax = bc::splat(0.f);
#pragma unroll
    for (int i = 0; i < fs::WAVES; ++i) tmax = (f2){fmaxf(tmax.x, red[2 * i]), fmaxf(tmax.y, red[2 * i + 1])};
    float* kred = red + 2 * fs::WAVES;
    const int coff = hp * 4;
    const f2 qscale = bc::splat(a.scale * kLog2e);
    float vabs = 0.f;
    int staged = -1;
    const int slots = cnt * H;
    for (int s0 = 0; s0 < slots; s0 += fs::WAVES * 64) {
        const int whi = (s0 + fs::WAVES * 64 - 1) / H < cnt - 1 ? (s0 + fs::WAVES * 64 - 1) / H : cnt - 1;
        for (int wi = staged + 1; wi <= whi; ++wi) {   // stage the round's new windows
            const int w = xcd + 8 * (j0 + wi);
            char* rs = ring + (wi % fs::RING) * fs::SLOT;
            f2 kn = bc::splat(0.f);
            if (tid < H) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const TokenInfo ti = token_info(g, w, tid + u * H);
                    const float4 kr = *reinterpret_cast<const float4*>(a.k + ti.row * a.ks + coff);
                    const float4 vr = *reinterpret_cast<const float4*>(a.v + ti.row * a.vs + coff);
                    kn = (f2){fmaxf(kn.x, kr.x * kr.x + kr.y * kr.y), fmaxf(kn.y, kr.z * kr.z + kr.w * kr.w)};
                    vabs = fmaxf(vabs, fmaxf(fmaxf(fabsf(vr.x), fabsf(vr.y)), fmaxf(fabsf(vr.z), fabsf(vr.w))));
                    f2* kv2 = reinterpret_cast<f2*>(rs) + tid * 8 + u * 4;
                    kv2[0] = (f2){kr.x, kr.z};
                    kv2[1] = (f2){kr.y, kr.w};
                    kv2[2] = (f2){vr.x, vr.z};
                    kv2[3] = (f2){vr.y, vr.w};
                }
            }
            if (wave < 2) {   // the staging threads are waves 0 and 1
                for (int off = 1; off < 64; off <<= 1)
                    kn = (f2){fmaxf(kn.x, __shfl_xor(kn.x, off)), fmaxf(kn.y, __shfl_xor(kn.y, off))};
                if (lane == 0) {
                    kred[((wi % fs::RING) * 2 + wave) * 2] = kn.x;
                    kred[((wi % fs::RING) * 2 + wave) * 2 + 1] = kn.y;
                }
            }
        }
        staged = whi > staged ? whi : staged;
        __syncthreads();   // the round's records and bounds are in LDS
        const int sl = s0 + tid;
        const bool active = sl < slots;
        const int wi = active ? sl / H : 0, pr = active ? sl - (sl / H) * H : 0;
        const int w = xcd + 8 * (j0 + wi);
        const int t = (int)bc::kPerm666[pr];
        const int rslot = wi % fs::RING;
        const bc::Regions reg = bc::window_regions(g, w);
        Row q[2], o[2];
        f2 m[2], l[2];
        int cq = 0, rq[2] = {0, 0};
        int64_t row[2] = {0, 0};
        bool rows_ok = true;
        if (active) {
            const f2 kmax2 = (f2){fmaxf(kred[rslot * 4], kred[rslot * 4 + 2]), fmaxf(kred[rslot * 4 + 1], kred[rslot * 4 + 3])};
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int tt = t + u * H;
                const TokenInfo ti = token_info(g, w, tt);
                row[u] = ti.row;
                rq[u] = bc::region_code(reg, tt / (WW * WH), (tt / WW) % WH, tt % WW);
                if (u == 0) cq = ti.code + Wn::OFF;
                q[u] = bc::load_row_pk(a.q + ti.row * a.qs + coff);
                q[u].x[0] *= qscale;
                q[u].x[1] *= qscale;
                l[u] = bc::splat(0.f);
                o[u].x[0] = o[u].x[1] = bc::splat(0.f);
                const f2 qn = bc::pfma(q[u].x[0], q[u].x[0], q[u].x[1] * q[u].x[1]);
                const f2 qk = qn * kmax2;
                rows_ok = rows_ok && __builtin_sqrtf(qk.x) + tmax.x <= kFwdBound &&
                          __builtin_sqrtf(qk.y) + tmax.y <= kFwdBound;
            }
        }
        const bool bounded = __all(rows_ok);
        const bool masked = __any(active && reg.masked);   // the masked loop is exact for any window
        const float* kv = reinterpret_cast<const float*>(ring + rslot * fs::SLOT);
        if (active) {
            if (bounded) {
                if (masked) fwd_loop<WD, WH, WW, true, true>(q, m, l, o, cq, rq, reg, tab_s, kv);
                else fwd_loop<WD, WH, WW, false, true>(q, m, l, o, cq, rq, reg, tab_s, kv);
            } else {
                if (masked) fwd_loop<WD, WH, WW, true, false>(q, m, l, o, cq, rq, reg, tab_s, kv);
                else fwd_loop<WD, WH, WW, false, false>(q, m, l, o, cq, rq, reg, tab_s, kv);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const f2 inv = (f2){1.0f / l[u].x, 1.0f / l[u].y};
                Row r;
                r.x[0] = o[u].x[0] * inv;
                r.x[1] = o[u].x[1] * inv;
                bc::store_row_nat(a.out + row[u] * a.os + coff, r, 1.0f);
                a.lse[row[u] * NHT + 2 * hp] = (m[u].x + fast_log2(l[u].x)) * kLn2;
                a.lse[row[u] * NHT + 2 * hp + 1] = (m[u].y + fast_log2(l[u].y)) * kLn2;
            }
        }
        __syncthreads();   // the round's record reads are done before the next round restages
    }
    if (a.vmax != nullptr) {
        for (int off = 32; off > 0; off >>= 1) vabs = fmaxf(vabs, __shfl_xor(vabs, off));
        if (lane == 0) atomicMax(a.vmax, __float_as_uint(vabs));
    }
}


// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
// The broadcast backward covers kind 0, head_dim 2, an even head count and the compiled window
// shapes (6^3: the C3 geometry).
bool wattn_bc_supported(const WGeom& g, int C, int heads, int kind) {
    if (kind != 0 || C != 2 * heads || heads % 2 != 0) return false;
    return g.wd == 6 && g.wh == 6 && g.ww == 6;
}


// merged backward: per_cu resident 4-wave workgroups per CU (2 by LDS), a multiple of 8 with every
// head pair served
static int q4_blocks(int per_cu, int NHG) {
    int grid = per_cu * kNumCU;
    grid -= grid % 8;
    return grid < 8 * NHG ? 8 * NHG : grid;
}

size_t wattn_bc_workspace_bytes(const WGeom& g, int heads) {
    const int grid = q4_blocks(2, heads / 2);
    return ((size_t)grid + 1) * g.Tsz * heads * sizeof(float);
}

static int set_lds_limit(const void* fn, size_t bytes) {
    if (bytes <= 64 * 1024) return 0;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) {
        set_error("hipFuncSetAttribute: %s", hipGetErrorString(e));
        return (int)e;
    }
    return 0;
}


int wattn_bc_forward(WAArgs& a, int heads, hipStream_t s) {
    const WGeom& g = a.g;
    constexpr int kTsz666 = bc::Win<6, 6, 6>::TSZ;
    MMNI_ARG_CHECK(g.wd == 6 && g.wh == 6 && g.ww == 6 && g.Tsz == kTsz666, "wattn_fwd (broadcast): compiled for 6^3 windows");
    const int NHG = heads / 2;
    a.hsplit = NHG;
    // forward with streaming lanes (all 256 lanes of a workgroup busy), 4 waves per SIMD
    const size_t lds = (size_t)bc::align4(kTsz666 * 2) * 4 + (size_t)fs::RING * fs::SLOT +
                       (size_t)(2 * fs::WAVES + 4 * fs::RING) * 4;
    int per = (4 * kNumCU) / (8 * NHG);   // 4-wave workgroups per CU (one per wave/SIMD)
    if (per < 1) per = 1;
    wattn_fwd_bcs_kernel<6, 6, 6><<<8 * NHG * per, fs::WAVES * 64, lds, s>>>(a);
    return launch_status("wattn_fwd_bcs");
}

int wattn_bc_backward(WAArgs& a, int heads, float* dtable, void* workspace, hipStream_t s) {
    const WGeom& g = a.g;
    constexpr int kTsz666 = bc::Win<6, 6, 6>::TSZ;
    MMNI_ARG_CHECK(g.wd == 6 && g.wh == 6 && g.ww == 6 && g.Tsz == kTsz666, "wattn_bwd (broadcast): compiled for 6^3 windows");
    const int NHG = heads / 2;
    a.hsplit = NHG;
    const int grid = q4_blocks(2, NHG);
    int rc = set_lds_limit(reinterpret_cast<const void*>(&wattn_bwd_q4k_kernel), k4::LDS);
    if (rc) return rc;
    const int ncol = g.Tsz * heads;
    float* part = static_cast<float*>(workspace);          // [grid][Tsz * heads]
    wattn_bwd_q4k_kernel<<<grid, k4::WAVES * 64, k4::LDS, s>>>(a, part);
    rc = launch_status("wattn_bwd_q4k");
    if (rc) return rc;
    ColSegs segs{};   // dtable += the fixed-order column sums of the workgroups' partial rows
    segs.n = 1;
    segs.end[0] = ncol;
    segs.dst[0] = dtable;
    segs.accumulate = 1;
    column_sum_segs(part, grid, ncol, segs, s);
    return launch_status("wattn_bwd_dtable_sum");
}

}  // namespace mmni
