// Window-attention backward for head_dim 2, "row-broadcast" formulation (SURVEY §8 rows a1, a3;
// reference: WindowAttention_fusion.forward swinfusion_module.py:114-145 and
// Cross_WindowAttention.forward :213-246, whose autograd backward this replaces).
//
// Two kernels per call, one workgroup = one (window, head pair) at a time, persistent:
//   pass A  (wattn_bwdA_bc_kernel)  lane = query pair (t, t + N/2)  ->  dq and the bias-table gradient
//   pass B  (wattn_bwdB_bc_kernel)  lane = key pair   (t, t + N/2)  ->  dk and dv
// Every lane of a wave walks the SAME other-side row pair at each step (keys in pass A, queries in
// pass B): those rows are LDS broadcast reads, and the per-lane work per (query, key, head pair)
// is the bare recompute + gradient on packed fp32: no online reductions, no cross-lane traffic.
//
// LDS facts that shape it (measured here, gfx950): a same-address ds_read_b128 does NOT broadcast
// (it ran ~16x slower than 8-byte broadcasts), so broadcast rows are stored as 8-byte component
// arrays ([component][row] f2) read by ds_read_b64 / ds_read2_b64.  The window is a compile-time shape (6^3 at the C3 geometry), so
// the key/query coordinates and codes are scalar loop counters, and every table access of a step
// is one address register plus immediate offsets.
//
// Bias-table gradient without atomics.  At one step the wave's lanes hold distinct queries against
// the same key pair, so the relative-position entries they update, code(q) - code(k) + off, are
// pairwise distinct (with the paired rows: entries E0, E0 - d, E0 + d, d = code(N/2), and no two
// lanes' sets intersect because no two of their queries are N/2 apart).  Each wave therefore
// read-modify-writes its OWN fp32 copy of the table in LDS with plain loads and stores: no atomics,
// no fixed-point scale, no max|dO| pre-pass.  A workgroup always serves the same head pair; its
// waves' copies are summed in a fixed order at the end into one partial row per workgroup, and a
// fixed-order column sum (tokenops.hip) adds the rows: bitwise deterministic.
//
// Kind 0 only (scaled dot + table bias), one head pair (4 channels) per workgroup, windows with an
// even first extent (N/2 = whole planes).
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

// (window, head pair) items: the NHG head-pair workgroups of a window sit 8 block indices apart,
// i.e. on one XCD (blocks are dealt round-robin over the 8 XCDs), so a window's rows are fetched
// from HBM once into that XCD's L2.  The grid is a multiple of 8 * NHG.
struct Items {
    int hp, first, stride;
};

__device__ __forceinline__ Items items(int NHG) {
    Items it;
    const int xslot = blockIdx.x >> 3;
    it.hp = xslot % NHG;
    it.first = (xslot / NHG) * 8 + (blockIdx.x & 7);
    it.stride = gridDim.x / NHG;
    return it;
}

constexpr int kThreads = 128;   // two waves: N / 2 <= 128 row pairs

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
// pass A: lane = query pair (t, t + H); keys (n, n + H) broadcast; dq + private table gradient
// ------------------------------------------------------------------------------------
// LDS tables, TSZ entries of one f2 (the head pair) each: bias * log2 e, then wave 0's and wave
// 1's table gradients, TSZ * 8 B apart (beyond ds_read2_b64's reach: each access stays one
// ds_read_b64 / ds_write_b64), all addressed from one lane register plus immediates.
template <int WD, int WH, int WW, int WAVE, bool MASKED, bool FOLD>
__device__ __forceinline__ void bwdA_loop(const Row (&q)[2], const Row (&dO)[2], const f2 (&lse2)[2],
                                          const f2 (&ndl)[2], Row (&dq)[2], int cq, const int (&rq)[2],
                                          const bc::Regions& reg, float* tabdt, const float* kv_s) {
    using Wn = bc::Win<WD, WH, WW>;
    constexpr int EB = 8;                           // entry bytes
    constexpr int DTO = (1 + WAVE) * Wn::TSZ * EB;  // this wave's table gradient
    char* tb = reinterpret_cast<char*>(tabdt);
    // lane address of entry (cq - code(n) - DC) = E- for code(n) = 0; E0 / E+ at +DC / +2 DC entries
    const uint32_t lane_base = (uint32_t)((cq - Wn::DC) * EB);
    const f2* kv2 = reinterpret_cast<const f2*>(kv_s);
    // Software pipeline: the broadcast K/V rows and the (read-only) bias entries of key n + 1 are
    // loaded during key n.  The private-table read-modify-write is the one ordered access: lanes
    // share entries across consecutive keys (lane t at key n + 1 reads what lane t - 1 wrote at
    // key n), a cross-lane order the compiler cannot see, so a compiler barrier after each key's
    // table stores keeps every later table read behind them (LDS executes a wave's accesses in
    // order; no wait is needed).
    // Keys are walked row by row (a row = WW consecutive keys, fixed (i, j)).  Per row one uniform
    // base addresses the broadcast K/V records and one lane base the table entries, so every
    // per-key access below is a base register plus an immediate offset (no per-key address math):
    // record of key n at kv2[8 n] (k c0, k c1, v c0, v c1 of key n, then of key n + H); entries of
    // key k of the row at trow + (WW - 1 - k) EB, trow = lane_base - (code0 + WW - 1) EB.
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
    for (int i = 0; i < WD / 2; ++i) {
        for (int j = 0; j < WH; ++j) {
            const int code0 = i * Wn::TW + j * Wn::TH;
            const f2* kvr = kv2 + (i * WH + j) * WW * 8;
            char* trow = tb + (lane_base - (uint32_t)((code0 + WW - 1) * EB));
            // the next row's bases, for the prefetch at the row's last key (the final row re-reads
            // itself: valid, unused data)
            const int jn = j + 1 < WH ? j + 1 : 0, in = j + 1 < WH ? i : i + 1;
            const bool last = in == WD / 2;
            const f2* kvn = last ? kvr : kv2 + (in * WH + jn) * WW * 8;
            const char* pen = last ? trow : tb + (lane_base - (uint32_t)((in * Wn::TW + jn * Wn::TH) * EB));
#pragma unroll
            for (int k = 0; k < WW; ++k) {
                char* pm = trow + (WW - 1 - k) * EB;   // entry E-  (query t, key n + H)
                // this key's table-gradient entries (after the previous key's stores), read BEFORE
                // the next key's prefetch: LDS returns in order, so waiting for these then leaves
                // the prefetch in flight across the step
                f2* dm = reinterpret_cast<f2*>(pm + DTO);
                f2* d0 = reinterpret_cast<f2*>(pm + Wn::DC * EB + DTO);
                f2* dp = reinterpret_cast<f2*>(pm + 2 * Wn::DC * EB + DTO);
                const f2 om = *dm, o0 = *d0, op = *dp;
                f2 nk[2][2], nv[2][2], nm, nz, np;
                if (k + 1 < WW) fetch(kvr + (k + 1) * 8, trow + (WW - 2 - k) * EB, nk, nv, nm, nz, np);
                else fetch(kvn, pen, nk, nv, nm, nz, np);
                int rk[2] = {0, 0};
                if (MASKED) {
                    rk[0] = bc::region_code(reg, i, j, k);
                    rk[1] = bc::region_code(reg, i + WD / 2, j, k);
                }
                f2 ds[2][2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
#pragma unroll
                    for (int v = 0; v < 2; ++v) {
                        const f2 t = (u == v) ? tb0 : (u == 0 ? tbm : tbp);
                        f2 base = FOLD ? t : t - lse2[u];   // FOLD: 2^-lse rides in dO and -delta
                        if (MASKED) base += bc::splat(rk[v] == rq[u] ? 0.f : kMask2);
                        f2 s = bc::pfma(q[u].x[0], kk[v][0], base);
                        s = bc::pfma(q[u].x[1], kk[v][1], s);
                        const f2 p = bc::exp2_2(s);
                        f2 tt = bc::pfma(dO[u].x[0], vv[v][0], ndl[u]);
                        tt = bc::pfma(dO[u].x[1], vv[v][1], tt);
                        ds[u][v] = p * tt;
                        dq[u].x[0] = bc::pfma(ds[u][v], kk[v][0], dq[u].x[0]);
                        dq[u].x[1] = bc::pfma(ds[u][v], kk[v][1], dq[u].x[1]);
                    }
                }
                // private table: no two lanes of the wave share an entry at one key
                *d0 = o0 + (ds[0][0] + ds[1][1]);
                *dm = om + ds[0][1];
                *dp = op + ds[1][0];
                asm volatile("" ::: "memory");
#pragma unroll
                for (int v = 0; v < 2; ++v)
#pragma unroll
                    for (int c = 0; c < 2; ++c) { kk[v][c] = nk[v][c]; vv[v][c] = nv[v][c]; }
                tbm = nm;
                tb0 = nz;
                tbp = np;
            }
        }
    }
}

template <int WD, int WH, int WW>
__global__ __launch_bounds__(bc::kThreads) __attribute__((amdgpu_waves_per_eu(2)))
void wattn_bwdA_bc_kernel(WAArgs a, float* part) {
    using Wn = bc::Win<WD, WH, WW>;
    constexpr int H = Wn::H, TSZ = Wn::TSZ;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int NHG = a.hsplit, NHT = 2 * NHG;
    float* tabdt = smem;                          // [3][TSZ] f2: bias pair, dt wave 0, dt wave 1
    float* kv_s = tabdt + bc::align4(TSZ * 6);    // [H][8] f2: k c0, k c1, v c0, v c1 of key n, then of n + H
    const bc::Items it = bc::items(NHG);
    const int tid = threadIdx.x, wave = tid >> 6;
    const bool lane_ok = tid < H;
    const int t = lane_ok ? (int)bc::kPerm666[tid] : 0;
    for (int e = tid; e < TSZ * 2; e += blockDim.x) {
        tabdt[e] = a.table[(e >> 1) * NHT + 2 * it.hp + (e & 1)] * kLog2e;
        tabdt[TSZ * 2 + e] = 0.f;
        tabdt[TSZ * 4 + e] = 0.f;
    }
    const int coff = it.hp * 4;
    const f2 qscale = bc::splat(a.scale * kLog2e);
    for (int w = it.first; w < g.nwin; w += it.stride) {
        __syncthreads();   // previous window's K/V reads done (and the table staged, first time)
        Row q[2], dO[2], dq[2];
        f2 lse2[2], ndl[2];
        int cq = 0, rq[2] = {0, 0};
        int64_t row[2] = {0, 0};
        const bc::Regions reg = bc::window_regions(g, w);
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int tt = t + u * H;
                const TokenInfo ti = token_info(g, w, tt);
                row[u] = ti.row;
                rq[u] = bc::region_code(reg, tt / (WW * WH), (tt / WW) % WH, tt % WW);
                if (u == 0) cq = ti.code + Wn::OFF;
                const float4 kr = *reinterpret_cast<const float4*>(a.k + ti.row * a.ks + coff);
                const float4 vr = *reinterpret_cast<const float4*>(a.v + ti.row * a.vs + coff);
                q[u] = bc::load_row_pk(a.q + ti.row * a.qs + coff);
                dO[u] = bc::load_row_pk(a.dout + ti.row * a.os + coff);
                const Row o = bc::load_row_pk(a.o + ti.row * a.os + coff);
                q[u].x[0] *= qscale;
                q[u].x[1] *= qscale;
                ndl[u] = -bc::pfma(o.x[0], dO[u].x[0], o.x[1] * dO[u].x[1]);
                lse2[u] = (f2){a.lse[ti.row * NHT + 2 * it.hp], a.lse[ti.row * NHT + 2 * it.hp + 1]} * kLog2e;
                f2* kv2 = reinterpret_cast<f2*>(kv_s) + t * 8 + u * 4;   // key record t
                kv2[0] = (f2){kr.x, kr.z};
                kv2[1] = (f2){kr.y, kr.w};
                kv2[2] = (f2){vr.x, vr.z};
                kv2[3] = (f2){vr.y, vr.w};
                dq[u].x[0] = dq[u].x[1] = bc::splat(0.f);
            }
        }
        __syncthreads();
        // the lane's rows are its own: the fold is decided per wave (uniform control flow)
        const bool fold = __all(!lane_ok || (bc::fold_ok(lse2[0]) && bc::fold_ok(lse2[1])));
        if (lane_ok) {
            if (fold) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const f2 e = bc::exp2_2(-lse2[u]);
                    dO[u].x[0] *= e;
                    dO[u].x[1] *= e;
                    ndl[u] *= e;
                }
            }
#define MMNI_BWDA(W, M, F) bwdA_loop<WD, WH, WW, W, M, F>(q, dO, lse2, ndl, dq, cq, rq, reg, tabdt, kv_s)
            if (fold) {
                if (reg.masked) {
                    if (wave == 0) MMNI_BWDA(0, true, true);
                    else MMNI_BWDA(1, true, true);
                } else {
                    if (wave == 0) MMNI_BWDA(0, false, true);
                    else MMNI_BWDA(1, false, true);
                }
            } else {
                if (reg.masked) {
                    if (wave == 0) MMNI_BWDA(0, true, false);
                    else MMNI_BWDA(1, true, false);
                } else {
                    if (wave == 0) MMNI_BWDA(0, false, false);
                    else MMNI_BWDA(1, false, false);
                }
            }
#undef MMNI_BWDA
#pragma unroll
            for (int u = 0; u < 2; ++u) bc::store_row_nat(a.dq + row[u] * a.qs + coff, dq[u], a.scale);
        }
    }
    __syncthreads();
    // this workgroup's partial row: its head pair's columns (wave 0 + wave 1, fixed order), zeros in
    // the other head pairs' columns
    float* prow = part + (int64_t)blockIdx.x * TSZ * NHT;
    for (int e = tid; e < TSZ * NHT; e += blockDim.x) {
        const int r = e / NHT, c = e - r * NHT;
        float v = 0.f;
        if ((c >> 1) == it.hp) v = tabdt[TSZ * 2 + r * 2 + (c & 1)] + tabdt[TSZ * 4 + r * 2 + (c & 1)];
        prow[e] = v;
    }
}

// ------------------------------------------------------------------------------------
// pass B: lane = key pair (t, t + H); queries (n, n + H) broadcast; dk, dv
// ------------------------------------------------------------------------------------
template <int WD, int WH, int WW, bool MASKED, bool FOLD>
__device__ __forceinline__ void bwdB_loop(const Row (&kr)[2], const Row (&vr)[2], Row (&dk)[2], Row (&dv)[2],
                                          int ck, const int (&rk)[2], const bc::Regions& reg, const float* tab_s,
                                          const float* rs_s) {
    using Wn = bc::Win<WD, WH, WW>;
    constexpr int EB = 8;
    const char* tb = reinterpret_cast<const char*>(tab_s);
    // entry of (query n, key t) = code(n) + ck, ck = OFF - code(t); (n, t + H) is DC lower,
    // (n + H, t) DC higher
    const uint32_t lane_base = (uint32_t)((ck - Wn::DC) * EB);
    // query records rs2[12 n]: q2 c0, q2 c1, dO c0, dO c1 of query n, the same of n + H, then -delta
    // of n and n + H, lse2 of n and n + H (16-byte groups);
    // per row one base each for the records and the table entries, immediates per query
    const f2* rs2 = reinterpret_cast<const f2*>(rs_s);
    for (int i = 0; i < WD / 2; ++i) {
        for (int j = 0; j < WH; ++j) {
            const int code0 = i * Wn::TW + j * Wn::TH;
            const f2* rsr = rs2 + (i * WH + j) * WW * 12;
            const char* trow = tb + (lane_base + (uint32_t)(code0 * EB));
#pragma unroll 3   // fully unrolled, the hoisted record loads spill at the 3-wave budget
            for (int k = 0; k < WW; ++k) {
                const char* pm = trow + k * EB;   // (n, t + H)
                f2 qq[2][2], gg[2][2], ls[2], nd[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const f2* src = rsr + k * 12 + u * 4;
                    bc::ld_pair(src, qq[u][0], qq[u][1]);
                    bc::ld_pair(src + 2, gg[u][0], gg[u][1]);
                }
                bc::ld_pair(rsr + k * 12 + 8, nd[0], nd[1]);
                if (FOLD) ls[0] = ls[1] = bc::splat(0.f);
                else bc::ld_pair(rsr + k * 12 + 10, ls[0], ls[1]);
                const f2 tbm = *reinterpret_cast<const f2*>(pm);
                const f2 tb0 = *reinterpret_cast<const f2*>(pm + Wn::DC * EB);
                const f2 tbp = *reinterpret_cast<const f2*>(pm + 2 * Wn::DC * EB);
                int rq[2] = {0, 0};
                if (MASKED) {
                    rq[0] = bc::region_code(reg, i, j, k);
                    rq[1] = bc::region_code(reg, i + WD / 2, j, k);
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {       // query n + u H
#pragma unroll
                    for (int v = 0; v < 2; ++v) {   // key t + v H
                        const f2 t = (u == v) ? tb0 : (u == 0 ? tbm : tbp);
                        f2 base = FOLD ? t : t - ls[u];
                        if (MASKED) base += bc::splat(rq[u] == rk[v] ? 0.f : kMask2);
                        f2 s = bc::pfma(qq[u][0], kr[v].x[0], base);
                        s = bc::pfma(qq[u][1], kr[v].x[1], s);
                        const f2 p = bc::exp2_2(s);
                        f2 tt = bc::pfma(gg[u][0], vr[v].x[0], nd[u]);
                        tt = bc::pfma(gg[u][1], vr[v].x[1], tt);
                        const f2 dsv = p * tt;
                        dv[v].x[0] = bc::pfma(p, gg[u][0], dv[v].x[0]);
                        dv[v].x[1] = bc::pfma(p, gg[u][1], dv[v].x[1]);
                        dk[v].x[0] = bc::pfma(dsv, qq[u][0], dk[v].x[0]);
                        dk[v].x[1] = bc::pfma(dsv, qq[u][1], dk[v].x[1]);
                    }
                }
            }
        }
    }
}

template <int WD, int WH, int WW>
__global__ __launch_bounds__(bc::kThreads) __attribute__((amdgpu_waves_per_eu(3)))
void wattn_bwdB_bc_kernel(WAArgs a) {
    using Wn = bc::Win<WD, WH, WW>;
    constexpr int H = Wn::H, TSZ = Wn::TSZ;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int NHG = a.hsplit, NHT = 2 * NHG;
    float* tab_s = smem;                            // [TSZ][2] bias * log2e of the head pair
    float* rs_s = tab_s + bc::align4(TSZ * 2);      // [H][12] f2: (q2 c0, q2 c1, dO c0, dO c1) x 2, -delta x 2, lse2 x 2
    const bc::Items it = bc::items(NHG);
    const int tid = threadIdx.x;
    const bool lane_ok = tid < H;
    const int t = lane_ok ? (int)bc::kPerm666[tid] : 0;
    for (int e = tid; e < TSZ * 2; e += blockDim.x) tab_s[e] = a.table[(e >> 1) * NHT + 2 * it.hp + (e & 1)] * kLog2e;
    const int coff = it.hp * 4;
    const float qs2 = a.scale * kLog2e;
    for (int w = it.first; w < g.nwin; w += it.stride) {
        Row kr[2], vr[2], dk[2], dv[2];
        int ck = 0, rk[2] = {0, 0};
        int64_t row[2] = {0, 0};
        const bc::Regions reg = bc::window_regions(g, w);
        TokenInfo ti[2];
        f2 l2[2] = {bc::splat(0.f), bc::splat(0.f)};
        bool bad = false;
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                ti[u] = token_info(g, w, t + u * H);
                l2[u] = (f2){a.lse[ti[u].row * NHT + 2 * it.hp], a.lse[ti[u].row * NHT + 2 * it.hp + 1]} * kLog2e;
                bad |= !bc::fold_ok(l2[u]);
            }
        }
        // every wave reads every query record: the fold is decided per window (this barrier also
        // orders the previous window's record reads before the stores below)
        const bool fold = !__syncthreads_or(bad);
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int tt = t + u * H;
                row[u] = ti[u].row;
                rk[u] = bc::region_code(reg, tt / (WW * WH), (tt / WW) % WH, tt % WW);
                if (u == 0) ck = Wn::OFF - ti[u].code;
                kr[u] = bc::load_row_pk(a.k + ti[u].row * a.ks + coff);
                vr[u] = bc::load_row_pk(a.v + ti[u].row * a.vs + coff);
                dk[u].x[0] = dk[u].x[1] = dv[u].x[0] = dv[u].x[1] = bc::splat(0.f);
                const float4 qr = *reinterpret_cast<const float4*>(a.q + ti[u].row * a.qs + coff);
                const float4 gr = *reinterpret_cast<const float4*>(a.dout + ti[u].row * a.os + coff);
                const float4 orow = *reinterpret_cast<const float4*>(a.o + ti[u].row * a.os + coff);
                const f2 e = fold ? bc::exp2_2(-l2[u]) : bc::splat(1.f);
                f2* rec = reinterpret_cast<f2*>(rs_s) + t * 12;   // query record t
                f2* dst = rec + u * 4;
                const float d0 = orow.x * gr.x + orow.y * gr.y, d1 = orow.z * gr.z + orow.w * gr.w;
                dst[0] = (f2){qr.x * qs2, qr.z * qs2};
                dst[1] = (f2){qr.y * qs2, qr.w * qs2};
                dst[2] = (f2){gr.x, gr.z} * e;
                dst[3] = (f2){gr.y, gr.w} * e;
                rec[8 + u] = (f2){-d0, -d1} * e;
                rec[10 + u] = l2[u];
            }
        }
        __syncthreads();
        if (lane_ok) {
            if (fold) {
                if (reg.masked) bwdB_loop<WD, WH, WW, true, true>(kr, vr, dk, dv, ck, rk, reg, tab_s, rs_s);
                else bwdB_loop<WD, WH, WW, false, true>(kr, vr, dk, dv, ck, rk, reg, tab_s, rs_s);
            } else {
                if (reg.masked) bwdB_loop<WD, WH, WW, true, false>(kr, vr, dk, dv, ck, rk, reg, tab_s, rs_s);
                else bwdB_loop<WD, WH, WW, false, false>(kr, vr, dk, dv, ck, rk, reg, tab_s, rs_s);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                bc::store_row_nat(a.dv + row[u] * a.vs + coff, dv[u], 1.0f);
                bc::store_row_nat(a.dk + row[u] * a.ks + coff, dk[u], kLn2);   // staged q2 = q * scale * log2e
            }
        }
    }
}

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

template <int WD, int WH, int WW>
__global__ __launch_bounds__(bc::kThreads) __attribute__((amdgpu_waves_per_eu(4)))
void wattn_fwd_bc_kernel(WAArgs a) {
    using Wn = bc::Win<WD, WH, WW>;
    constexpr int H = Wn::H, TSZ = Wn::TSZ;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const WGeom& g = a.g;
    const int NHG = a.hsplit, NHT = 2 * NHG;
    float* tab_s = smem;                 // [TSZ] f2: bias * log2e of the head pair
    float* kv_s = tab_s + bc::align4(TSZ * 2);   // [H][8] f2: key records as in pass A
    float* red = kv_s + H * 16;          // [2 waves][2 heads] max |bias|, then [2][2] max |k|^2
    const bc::Items it = bc::items(NHG);
    const int tid = threadIdx.x, wave = tid >> 6;
    const bool lane_ok = tid < H;
    const int t = lane_ok ? (int)bc::kPerm666[tid] : 0;
    float tabs = 0.f;   // this thread's entries all belong to head tid & 1 (the stride is even)
    for (int e = tid; e < TSZ * 2; e += blockDim.x) {
        const float x = a.table[(e >> 1) * NHT + 2 * it.hp + (e & 1)] * kLog2e;
        tab_s[e] = x;
        tabs = fmaxf(tabs, fabsf(x));
    }
    for (int off = 2; off < 64; off <<= 1) tabs = fmaxf(tabs, __shfl_xor(tabs, off));
    if ((tid & 63) < 2) red[wave * 2 + (tid & 1)] = tabs;
    __syncthreads();
    const f2 tmax = (f2){fmaxf(red[0], red[2]), fmaxf(red[1], red[3])};
    const int coff = it.hp * 4;
    const f2 qscale = bc::splat(a.scale * kLog2e);
    float vabs = 0.f;
    for (int w = it.first; w < g.nwin; w += it.stride) {
        __syncthreads();   // previous window's K/V reads done (and the table staged, first time)
        Row q[2], o[2];
        f2 m[2], l[2];
        int cq = 0, rq[2] = {0, 0};
        int64_t row[2] = {0, 0};
        const bc::Regions reg = bc::window_regions(g, w);
        f2 kn = bc::splat(0.f);   // max |k|^2 per head over this lane's two keys
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int tt = t + u * H;
                const TokenInfo ti = token_info(g, w, tt);
                row[u] = ti.row;
                rq[u] = bc::region_code(reg, tt / (WW * WH), (tt / WW) % WH, tt % WW);
                if (u == 0) cq = ti.code + Wn::OFF;
                const float4 kr = *reinterpret_cast<const float4*>(a.k + ti.row * a.ks + coff);
                const float4 vr = *reinterpret_cast<const float4*>(a.v + ti.row * a.vs + coff);
                q[u] = bc::load_row_pk(a.q + ti.row * a.qs + coff);
                q[u].x[0] *= qscale;
                q[u].x[1] *= qscale;
                kn = (f2){fmaxf(kn.x, kr.x * kr.x + kr.y * kr.y), fmaxf(kn.y, kr.z * kr.z + kr.w * kr.w)};
                vabs = fmaxf(vabs, fmaxf(fmaxf(fabsf(vr.x), fabsf(vr.y)), fmaxf(fabsf(vr.z), fabsf(vr.w))));
                f2* kv2 = reinterpret_cast<f2*>(kv_s) + t * 8 + u * 4;   // key record t
                kv2[0] = (f2){kr.x, kr.z};
                kv2[1] = (f2){kr.y, kr.w};
                kv2[2] = (f2){vr.x, vr.z};
                kv2[3] = (f2){vr.y, vr.w};
                l[u] = bc::splat(0.f);
                o[u].x[0] = o[u].x[1] = bc::splat(0.f);
            }
        }
        for (int off = 1; off < 64; off <<= 1)
            kn = (f2){fmaxf(kn.x, __shfl_xor(kn.x, off)), fmaxf(kn.y, __shfl_xor(kn.y, off))};
        if ((tid & 63) == 0) {
            red[4 + wave * 2] = kn.x;
            red[5 + wave * 2] = kn.y;
        }
        __syncthreads();
        // per wave: every row within the bound (the previous window's reads of red[4..7] finished
        // before this window's first barrier)
        const f2 kmax2 = (f2){fmaxf(red[4], red[6]), fmaxf(red[5], red[7])};
        bool rows_ok = true;
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const f2 qn = bc::pfma(q[u].x[0], q[u].x[0], q[u].x[1] * q[u].x[1]);
                const f2 qk = qn * kmax2;
                rows_ok = rows_ok && __builtin_sqrtf(qk.x) + tmax.x <= kFwdBound &&
                          __builtin_sqrtf(qk.y) + tmax.y <= kFwdBound;
            }
        }
        const bool bounded = __all(rows_ok);
        if (lane_ok) {
            if (bounded) {
                if (reg.masked) fwd_loop<WD, WH, WW, true, true>(q, m, l, o, cq, rq, reg, tab_s, kv_s);
                else fwd_loop<WD, WH, WW, false, true>(q, m, l, o, cq, rq, reg, tab_s, kv_s);
            } else {
                if (reg.masked) fwd_loop<WD, WH, WW, true, false>(q, m, l, o, cq, rq, reg, tab_s, kv_s);
                else fwd_loop<WD, WH, WW, false, false>(q, m, l, o, cq, rq, reg, tab_s, kv_s);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const f2 inv = (f2){1.0f / l[u].x, 1.0f / l[u].y};
                Row r;
                r.x[0] = o[u].x[0] * inv;
                r.x[1] = o[u].x[1] * inv;
                bc::store_row_nat(a.out + row[u] * a.os + coff, r, 1.0f);
                a.lse[row[u] * NHT + 2 * it.hp] = (m[u].x + fast_log2(l[u].x)) * kLn2;
                a.lse[row[u] * NHT + 2 * it.hp + 1] = (m[u].y + fast_log2(l[u].y)) * kLn2;
            }
        }
    }
    if (a.vmax != nullptr) {
        for (int off = 32; off > 0; off >>= 1) vabs = fmaxf(vabs, __shfl_xor(vabs, off));
        if ((tid & 63) == 0) atomicMax(a.vmax, __float_as_uint(vabs));
    }
}

// ------------------------------------------------------------------------------------
// "quad" layout of 6^3 windows: a lane owns the row quad {b, b + 18, b + 108, b + 126} (its
// (y + 3, z + 3) partners), b = (z', y', x) with z', y' < 3: 54 lanes = one wave per (window, head
// pair).  The wave walks the 54 key quads in lock step, so each broadcast record (4 keys x k, v)
// feeds 16 (query, key) pairs instead of 4, and the 16 pairs of a step touch only 9 table entries
// (relative offsets a * 3 TW + b * 3 TH, a, b in {-1, 0, 1}).  The bases' codes hit each of the 32
// 8-byte bank pairs once in lanes 0-31 and at most once in lanes 32-53 (kPermQ), so every
// per-lane table access is conflict-free.  The 9 x 54 entries of one step are pairwise distinct
// (codes of bases differ by less than 3 in every digit), so the private table read-modify-write
// of a step never aliases across lanes.
// ------------------------------------------------------------------------------------
#ifndef MMNI_Q4_DSADD
#define MMNI_Q4_DSADD 0   // table gradient by LDS float adds (ds_add_f32) instead of read-modify-write
#endif
namespace q4 {
constexpr int NB = 54;                              // row quads per window
constexpr int TW = 121, TH = 11, OFF = 665, TSZ = 1331;
constexpr int EB = 8;                               // table entry: f2 over the head pair
constexpr int DMIN = 3 * TW + 3 * TH + 5;           // 401: entry offsets D + DMIN - x are >= 0
constexpr int REC = 128;                            // key-quad record: 4 keys x (k f4, v f4)
constexpr int KVB = NB * REC;                       // 6912 B of records per wave
constexpr int WAVES = 4;                            // waves per workgroup (one head pair per workgroup)
constexpr int TABB = TSZ * EB;                      // 10648 B per table image
constexpr int TAB = WAVES * KVB;                    // bias table offset (records first: row bases >= 0)
constexpr int DT = (TAB + TABB + 15) & ~15;         // gradient images, one per wave
constexpr int LDS_A = DT + WAVES * TABB;            // 80896 B: two workgroups per CU
constexpr int LDS_F = TAB + TABB;                   // forward: records + bias table
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

template <bool MASKED, bool FOLD>
__device__ __forceinline__ void q4A_loop(const Row (&q)[4], const Row (&dO)[4], const f2 (&lse2)[4],
                                         const f2 (&ndl)[4], Row (&dq)[4], int lcode, const int (&rq)[4],
                                         const bc::Regions& reg, char* sm, int kvw, int dtw) {
    using namespace q4;
    const char* kv = sm + kvw;
    const char* tb = sm + TAB;
    // entry of combo slot e at key x of key row (zr, yr): row base + (D_e + DMIN - x) * EB,
    // row base = (lcode + OFF - DMIN - code0) * EB
    const uint32_t lane_e = (uint32_t)((lcode + OFF - DMIN) * EB);
    f2 kk[4][2], vv[4][2], bt[9];
    auto fetch = [&](const char* rec, const char* te, f2 (&k_)[4][2], f2 (&v_)[4][2], f2 (&b_)[9]) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            bc::ld_pair(reinterpret_cast<const f2*>(rec + v * 32), k_[v][0], k_[v][1]);
            bc::ld_pair(reinterpret_cast<const f2*>(rec + v * 32 + 16), v_[v][0], v_[v][1]);
        }
#pragma unroll
        for (int e = 0; e < 9; ++e) b_[e] = *reinterpret_cast<const f2*>(te + (dcode(e) + DMIN) * EB);
    };
    fetch(kv, tb + lane_e, kk, vv, bt);
    for (int zr = 0; zr < 3; ++zr) {
        for (int yr = 0; yr < 3; ++yr) {
            const uint32_t trow = lane_e - (uint32_t)((zr * TW + yr * TH) * EB);
            const char* tp = tb + trow;
            char* dp = sm + dtw + trow;
            const char* kvr = kv + (zr * 3 + yr) * 6 * REC;
            const int yn = yr + 1 < 3 ? yr + 1 : 0, zn = yr + 1 < 3 ? zr : zr + 1;
            const bool last = zn == 3;   // the final row's prefetch re-reads itself (unused)
            const char* kvn = last ? kvr : kv + (zn * 3 + yn) * 6 * REC;
            const char* tpn = last ? tp : tb + (lane_e - (uint32_t)((zn * TW + yn * TH) * EB));
#pragma unroll
            for (int x = 0; x < 6; ++x) {
                // this key quad's gradient entries, read before the next quad's prefetch (LDS
                // returns in order: waiting on these leaves the prefetch in flight)
                f2 od[9];
#if MMNI_Q4_DSADD
#pragma unroll
                for (int e = 0; e < 9; ++e) od[e] = bc::splat(0.f);
#else
#pragma unroll
                for (int e = 0; e < 9; ++e) od[e] = *reinterpret_cast<const f2*>(dp + (dcode(e) + DMIN - x) * EB);
#endif
                f2 nk[4][2], nv[4][2], nb[9];
                if (x + 1 < 6) fetch(kvr + (x + 1) * REC, tp - (x + 1) * EB, nk, nv, nb);
                else fetch(kvn, tpn, nk, nv, nb);
                int rk[4] = {0, 0, 0, 0};
                if (MASKED) {
#pragma unroll
                    for (int v = 0; v < 4; ++v) rk[v] = bc::region_code(reg, zr + 3 * (v >> 1), yr + 3 * (v & 1), x);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        const int e = slot(u, v);
                        f2 base = FOLD ? bt[e] : bt[e] - lse2[u];   // FOLD: 2^-lse rides in dO and -delta
                        if (MASKED) base += bc::splat(rk[v] == rq[u] ? 0.f : kMask2);
                        f2 s = bc::pfma(q[u].x[0], kk[v][0], base);
                        s = bc::pfma(q[u].x[1], kk[v][1], s);
                        const f2 p = bc::exp2_2(s);
                        f2 tt = bc::pfma(dO[u].x[0], vv[v][0], ndl[u]);
                        tt = bc::pfma(dO[u].x[1], vv[v][1], tt);
                        const f2 ds = p * tt;
                        dq[u].x[0] = bc::pfma(ds, kk[v][0], dq[u].x[0]);
                        dq[u].x[1] = bc::pfma(ds, kk[v][1], dq[u].x[1]);
                        od[e] += ds;
                    }
                }
#if MMNI_Q4_DSADD
#pragma unroll
                for (int e = 0; e < 9; ++e) {
                    float* pe = reinterpret_cast<float*>(dp + (dcode(e) + DMIN - x) * EB);
                    __hip_atomic_fetch_add(pe, od[e].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(pe + 1, od[e].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#else
#pragma unroll
                for (int e = 0; e < 9; ++e) *reinterpret_cast<f2*>(dp + (dcode(e) + DMIN - x) * EB) = od[e];
                asm volatile("" ::: "memory");   // the next quad's entry reads stay behind these stores
#endif
#pragma unroll
                for (int v = 0; v < 4; ++v)
#pragma unroll
                    for (int c = 0; c < 2; ++c) { kk[v][c] = nk[v][c]; vv[v][c] = nv[v][c]; }
#pragma unroll
                for (int e = 0; e < 9; ++e) bt[e] = nb[e];
            }
        }
    }
}

// pass A, quad layout: 4 waves per workgroup, one head pair per workgroup, each wave one window at
// a time with its own key records and private table-gradient image; no block barrier in the loop
// (a wave reads only what it wrote; LDS runs a wave's accesses in order)
__global__ __launch_bounds__(q4::WAVES * 64) __attribute__((amdgpu_waves_per_eu(2)))
void wattn_bwdA_q4_kernel(WAArgs a, float* part) {
    using namespace q4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    char* sm = reinterpret_cast<char*>(smem);
    const WGeom& g = a.g;
    const int NHG = a.hsplit, NHT = 2 * NHG;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const Work wk = work(NHG, wave);
    float* tab = reinterpret_cast<float*>(sm + TAB);
    for (int e = tid; e < TSZ * 2; e += blockDim.x) tab[e] = a.table[(e >> 1) * NHT + 2 * wk.hp + (e & 1)] * kLog2e;
    float* dtf = reinterpret_cast<float*>(sm + DT);
    for (int e = tid; e < WAVES * TSZ * 2; e += blockDim.x) dtf[e] = 0.f;
    __syncthreads();
    const bool lane_ok = lane < NB;
    const int beta = lane_ok ? (int)kPermQ[lane] : 0;
    const int tb0 = base_token(beta), lcode = base_code(beta);
    const int bz = beta / 18, by = (beta / 6) % 3, bx = beta % 6;
    const int kvw = wave * KVB, dtw = DT + wave * TABB;
    const int coff = wk.hp * 4;
    const f2 qscale = bc::splat(a.scale * kLog2e);
    for (int j = wk.j0;; j += wk.dj) {
        const int w = wk.xcd + 8 * j;
        if (w >= g.nwin) break;
        Row q[4], dO[4], dq[4];
        f2 lse2[4], ndl[4];
        int rq[4] = {0, 0, 0, 0};
        int64_t row[4] = {0, 0, 0, 0};
        const bc::Regions reg = bc::window_regions(g, w);
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const TokenInfo ti = token_info(g, w, tb0 + (u & 1) * 18 + (u >> 1) * 108);
                row[u] = ti.row;
                rq[u] = bc::region_code(reg, bz + 3 * (u >> 1), by + 3 * (u & 1), bx);
                const float4 kr = *reinterpret_cast<const float4*>(a.k + ti.row * a.ks + coff);
                const float4 vr = *reinterpret_cast<const float4*>(a.v + ti.row * a.vs + coff);
                q[u] = bc::load_row_pk(a.q + ti.row * a.qs + coff);
                dO[u] = bc::load_row_pk(a.dout + ti.row * a.os + coff);
                const Row o = bc::load_row_pk(a.o + ti.row * a.os + coff);
                q[u].x[0] *= qscale;
                q[u].x[1] *= qscale;
                ndl[u] = -bc::pfma(o.x[0], dO[u].x[0], o.x[1] * dO[u].x[1]);
                lse2[u] = (f2){a.lse[ti.row * NHT + 2 * wk.hp], a.lse[ti.row * NHT + 2 * wk.hp + 1]} * kLog2e;
                char* rec = sm + kvw + beta * REC + u * 32;   // key u of quad beta
                *reinterpret_cast<bc::f4*>(rec) = (bc::f4){kr.x, kr.z, kr.y, kr.w};
                *reinterpret_cast<bc::f4*>(rec + 16) = (bc::f4){vr.x, vr.z, vr.y, vr.w};
                dq[u].x[0] = dq[u].x[1] = bc::splat(0.f);
            }
        }
        asm volatile("" ::: "memory");   // the records are written before the walk reads them
        bool ok = true;
#pragma unroll
        for (int u = 0; u < 4; ++u) ok = ok && bc::fold_ok(lse2[u]);
        const bool fold = __all(!lane_ok || ok);
        if (lane_ok) {
            if (fold) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const f2 e = bc::exp2_2(-lse2[u]);
                    dO[u].x[0] *= e;
                    dO[u].x[1] *= e;
                    ndl[u] *= e;
                }
            }
#define MMNI_Q4A(M, F) q4A_loop<M, F>(q, dO, lse2, ndl, dq, lcode, rq, reg, sm, kvw, dtw)
            if (fold) {
                if (reg.masked) MMNI_Q4A(true, true);
                else MMNI_Q4A(false, true);
            } else {
                if (reg.masked) MMNI_Q4A(true, false);
                else MMNI_Q4A(false, false);
            }
#undef MMNI_Q4A
#pragma unroll
            for (int u = 0; u < 4; ++u) bc::store_row_nat(a.dq + row[u] * a.qs + coff, dq[u], a.scale);
        }
        asm volatile("" ::: "memory");   // the next window's records stay behind this walk's reads
    }
    __syncthreads();
    // this workgroup's partial row: its head pair's columns (waves 0..3 summed in order), zeros elsewhere
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
// merged backward, quad layout: pass A's walk (lane = query quad, key quads broadcast) also forms
// the key side.  Per step a lane holds, for the 4 keys of the quad, its partial dk and dv over its
// 4 query rows: 32 floats = 16 f2 over the head pair, value i = kind * 16 + v * 4 + c * 2 + h
// (kind 0 dk, 1 dv; key v, dim c, head h).  A fixed butterfly over the 64 lanes (v_permlane32_swap,
// v_permlane16_swap, then DPP row_ror:8 / row_half_mirror / quad xor 2 / xor 1) leaves lane l with
// the full sum of value l >> 1, which lane l (even) stores.  Every key quad is visited once per
// window, so those sums are final: no dk/dv accumulation, and p, ds are formed once per (query,
// key) instead of once in each pass.  Deterministic (fixed lane tree, fixed row order).
// ------------------------------------------------------------------------------------
#ifndef MMNI_Q4M_UNROLL
#define MMNI_Q4M_UNROLL 1   // unroll the merged walk's key loop
#endif
#ifndef MMNI_Q4M_PIPE
#define MMNI_Q4M_PIPE 0     // issue the next key quad's records during the lane reduction
#endif
namespace q4 {
// The spare lanes (54..63) of the merged walk run every step with zero dO, delta and q (so their
// ds and partials are exactly 0) and read-modify-write table entries at this code: 6 is no
// c_r + a * 3 TW + b * 3 TH (|a|, |b| <= 2) for any row-quad code c_r, so within one step their
// entries never meet a real lane's, and they write back the values they read.  No branch.
constexpr int kSpareCode = 6;
__constant__ unsigned char kInvPermQ[NB] = {0, 1, 2, 3, 4, 5, 11, 12, 13, 14, 15, 16, 22, 23, 24, 25, 26, 27, 32, 33, 34, 28, 29, 30, 35, 36, 6, 7, 8, 9, 37, 38, 17, 18, 19, 20, 39, 40, 41, 21, 42, 43, 44, 45, 31, 46, 47, 48, 49, 50, 10, 51, 52, 53};

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

// 16 f2 partials per lane -> lane l returns the 64-lane sum of value l >> 1
__device__ __forceinline__ float reduce32(f2 (&P)[16], int lane) {
    f2 R[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {   // lanes 0-31 keep f2 k (dk), lanes 32-63 f2 k + 8 (dv)
        float a0 = P[k].x, b0 = P[k + 8].x, a1 = P[k].y, b1 = P[k + 8].y;
        swap32(a0, b0);
        swap32(a1, b1);
        R[k] = (f2){a0, a1} + (f2){b0, b1};
    }
    f2 S[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {   // rows 0, 2 keep k (keys 0, 1), rows 1, 3 keep k + 4 (keys 2, 3)
        float a0 = R[k].x, b0 = R[k + 4].x, a1 = R[k].y, b1 = R[k + 4].y;
        swap16(a0, b0);
        swap16(a1, b1);
        S[k] = (f2){a0, a1} + (f2){b0, b1};
    }
    const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2;
    f2 T[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {   // lane bit 3: key 0 or 1 of the pair (row_ror:8 partner = lane ^ 8)
        const f2 keep = b3 ? S[k + 2] : S[k], send = b3 ? S[k] : S[k + 2];
        T[k] = keep + (f2){dpp<0x128>(send.x), dpp<0x128>(send.y)};
    }
    // lane bit 2: dim c (row_half_mirror partner = lane ^ 7 within 8)
    const f2 keep = b2 ? T[1] : T[0], send = b2 ? T[0] : T[1];
    const f2 U = keep + (f2){dpp<0x141>(send.x), dpp<0x141>(send.y)};
    // lane bit 1: head h (quad partner lane ^ 2), then lane ^ 1
    const float kv = b1 ? U.y : U.x, sv = b1 ? U.x : U.y;
    const float V = kv + dpp<0x4E>(sv);
    return V + dpp<0xB1>(V);
}
}  // namespace q4

template <bool MASKED, bool FOLD>
__device__ __forceinline__ void q4M_loop(const Row (&q)[4], const Row (&dO)[4], const f2 (&lse2)[4],
                                         const f2 (&ndl)[4], Row (&dq)[4], int lcode, const int (&rq)[4],
                                         const bc::Regions& reg, char* sm, int kvw, int dtw, bool lane_ok,
                                         const int (&rowk)[4], float* kout, int64_t kstride, float kscale) {
    using namespace q4;
    const int lane = threadIdx.x & 63;
    const char* kv = sm + kvw;
    const uint32_t lane_e = (uint32_t)((lcode + OFF - DMIN) * EB);
    const int vsel = (lane >> 3) & 3;   // the key whose sum this lane ends with (l >> 1 = kind, v, c, h)
    // MMNI_Q4M_PIPE: after a step's table stores, the next step's records and bias entries are
    // issued and the step's lane reduction (pure VALU) runs while they are in flight.  The table
    // base goes through an empty asm after the stores, so the compiler treats the next step's table
    // reads as possibly aliasing them (other lanes' entries) and keeps them behind the stores; LDS
    // executes a wave's accesses in order, so no wait is needed.
    f2 kk[4][2], vv[4][2], bt[9], od[9];
    auto load = [&](const char* rec, const char* te) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            bc::ld_pair(reinterpret_cast<const f2*>(rec + v * 32), kk[v][0], kk[v][1]);
            bc::ld_pair(reinterpret_cast<const f2*>(rec + v * 32 + 16), vv[v][0], vv[v][1]);
        }
#pragma unroll
        for (int e = 0; e < 9; ++e) bt[e] = *reinterpret_cast<const f2*>(te + (dcode(e) + DMIN) * EB);
    };
    int dto = dtw;   // this wave's table-gradient image (an LDS offset: the accesses stay ds_*)
    if (MMNI_Q4M_PIPE) load(kv, sm + TAB + lane_e);
    for (int zr = 0; zr < 3; ++zr) {
        for (int yr = 0; yr < 3; ++yr) {
            const uint32_t trow = lane_e - (uint32_t)((zr * TW + yr * TH) * EB);
            const int yn = yr + 1 < 3 ? yr + 1 : 0, zn = yr + 1 < 3 ? zr : zr + 1;
            const bool last = zn == 3;   // the final row's prefetch re-reads itself (unused)
            const uint32_t trown = last ? trow : lane_e - (uint32_t)((zn * TW + yn * TH) * EB);
            const char* kvr = kv + (zr * 3 + yr) * 6 * REC;
            const char* kvn = last ? kvr : kv + (zn * 3 + yn) * 6 * REC;
#pragma unroll
            for (int x = 0; x < 6; ++x) {
                // spare lanes skip the step (a divergent branch here measured spill-free; without it
                // the compiler spilled ~800 VGPRs) and contribute zero partials
                f2 P[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) P[i] = bc::splat(0.f);
                if (lane_ok) {
                    char* dp = sm + dto + trow;
                    // this step's table-gradient entries (after the previous step's stores: see dto)
#pragma unroll
                    for (int e = 0; e < 9; ++e) od[e] = *reinterpret_cast<const f2*>(dp + (dcode(e) + DMIN - x) * EB);
                    if (!MMNI_Q4M_PIPE) load(kvr + x * REC, sm + TAB + trow - x * EB);
                    int rk[4] = {0, 0, 0, 0};
                    if (MASKED) {
#pragma unroll
                        for (int v = 0; v < 4; ++v) rk[v] = bc::region_code(reg, zr + 3 * (v >> 1), yr + 3 * (v & 1), x);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
#pragma unroll
                        for (int v = 0; v < 4; ++v) {
                            const int e = slot(u, v);
                            f2 base = FOLD ? bt[e] : bt[e] - lse2[u];
                            if (MASKED) base += bc::splat(rk[v] == rq[u] ? 0.f : kMask2);
                            f2 s = bc::pfma(q[u].x[0], kk[v][0], base);
                            s = bc::pfma(q[u].x[1], kk[v][1], s);
                            const f2 p = bc::exp2_2(s);
                            f2 tt = bc::pfma(dO[u].x[0], vv[v][0], ndl[u]);
                            tt = bc::pfma(dO[u].x[1], vv[v][1], tt);
                            const f2 ds = p * tt;
                            dq[u].x[0] = bc::pfma(ds, kk[v][0], dq[u].x[0]);
                            dq[u].x[1] = bc::pfma(ds, kk[v][1], dq[u].x[1]);
                            od[e] += ds;
                            if (u == 0) {   // first row: plain products (P is zero)
                                P[v * 2] = ds * q[0].x[0];              // dk, dim 0
                                P[v * 2 + 1] = ds * q[0].x[1];          // dk, dim 1
                                P[8 + v * 2] = p * dO[0].x[0];          // dv, dim 0
                                P[8 + v * 2 + 1] = p * dO[0].x[1];      // dv, dim 1
                            } else {
                                P[v * 2] = bc::pfma(ds, q[u].x[0], P[v * 2]);
                                P[v * 2 + 1] = bc::pfma(ds, q[u].x[1], P[v * 2 + 1]);
                                P[8 + v * 2] = bc::pfma(p, dO[u].x[0], P[8 + v * 2]);
                                P[8 + v * 2 + 1] = bc::pfma(p, dO[u].x[1], P[8 + v * 2 + 1]);
                            }
                        }
                    }
#pragma unroll
                    for (int e = 0; e < 9; ++e) *reinterpret_cast<f2*>(dp + (dcode(e) + DMIN - x) * EB) = od[e];
                }
                asm volatile("" : "+v"(dto));   // next reads: behind the stores above (see the top)
                __builtin_amdgcn_sched_barrier(0);   // keep later steps' loads from being hoisted (registers)
                if (MMNI_Q4M_PIPE) {
                    if (x + 1 < 6) load(kvr + (x + 1) * REC, sm + TAB + trow - (x + 1) * EB);
                    else load(kvn, sm + TAB + trown);
                }
                // all 64 lanes take part in the reduction (spare lanes contribute zeros)
                const float sum = reduce32(P, lane);
                // rows of key quad n = (zr, yr, x): held by the lane that owns query quad n
                const int owner = kInvPermQ[(zr * 3 + yr) * 6 + x];
                const int r0 = __builtin_amdgcn_readlane(rowk[0], owner), r1 = __builtin_amdgcn_readlane(rowk[1], owner);
                const int r2 = __builtin_amdgcn_readlane(rowk[2], owner), r3 = __builtin_amdgcn_readlane(rowk[3], owner);
                const int r = vsel == 0 ? r0 : (vsel == 1 ? r1 : (vsel == 2 ? r2 : r3));
                if ((lane & 1) == 0) kout[(int64_t)r * kstride] = sum * kscale;
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
}

// merged backward: dq, dk, dv and the table gradient in one walk (4 waves per workgroup as pass A)
__global__ __launch_bounds__(q4::WAVES * 64) __attribute__((amdgpu_waves_per_eu(2)))
void wattn_bwd_q4m_kernel(WAArgs a, float* part) {
    using namespace q4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    char* sm = reinterpret_cast<char*>(smem);
    const WGeom& g = a.g;
    const int NHG = a.hsplit, NHT = 2 * NHG;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const Work wk = work(NHG, wave);
    float* tab = reinterpret_cast<float*>(sm + TAB);
    for (int e = tid; e < TSZ * 2; e += blockDim.x) tab[e] = a.table[(e >> 1) * NHT + 2 * wk.hp + (e & 1)] * kLog2e;
    float* dtf = reinterpret_cast<float*>(sm + DT);
    for (int e = tid; e < WAVES * TSZ * 2; e += blockDim.x) dtf[e] = 0.f;
    __syncthreads();
    const bool lane_ok = lane < NB;
    const int beta = lane_ok ? (int)kPermQ[lane] : 0;   // spare lanes run the walk on zero rows
    const int tb0 = base_token(beta), lcode = lane_ok ? base_code(beta) : kSpareCode;
    const int bz = beta / 18, by = (beta / 6) % 3, bx = beta % 6;
    const int kvw = wave * KVB, dtw = DT + wave * TABB;
    const int coff = wk.hp * 4;
    const f2 qscale = bc::splat(a.scale * kLog2e);
    // this lane's output slot of the key-side sums: value l >> 1 = (kind, key, dim c, head h)
    const bool is_dv = lane & 32;
    const int comp = ((lane >> 1) & 1) * 2 + ((lane >> 2) & 1);   // global row order (h0c0, h0c1, h1c0, h1c1)
    float* kout = (is_dv ? a.dv : a.dk) + coff + comp;
    const int64_t kstride = is_dv ? a.vs : a.ks;
    const float kscale = is_dv ? 1.0f : kLn2;   // dk: the staged q carries scale * log2 e
    for (int j = wk.j0;; j += wk.dj) {
        const int w = wk.xcd + 8 * j;
        if (w >= g.nwin) break;
        Row q[4], dO[4], dq[4];
        f2 lse2[4], ndl[4];
        int rq[4] = {0, 0, 0, 0}, rowk[4] = {0, 0, 0, 0};
        const bc::Regions reg = bc::window_regions(g, w);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            q[u].x[0] = q[u].x[1] = dO[u].x[0] = dO[u].x[1] = dq[u].x[0] = dq[u].x[1] = bc::splat(0.f);
            lse2[u] = ndl[u] = bc::splat(0.f);
        }
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const TokenInfo ti = token_info(g, w, tb0 + (u & 1) * 18 + (u >> 1) * 108);
                rowk[u] = (int)ti.row;
                rq[u] = bc::region_code(reg, bz + 3 * (u >> 1), by + 3 * (u & 1), bx);
                const float4 kr = *reinterpret_cast<const float4*>(a.k + ti.row * a.ks + coff);
                const float4 vr = *reinterpret_cast<const float4*>(a.v + ti.row * a.vs + coff);
                q[u] = bc::load_row_pk(a.q + ti.row * a.qs + coff);
                dO[u] = bc::load_row_pk(a.dout + ti.row * a.os + coff);
                const Row o = bc::load_row_pk(a.o + ti.row * a.os + coff);
                q[u].x[0] *= qscale;
                q[u].x[1] *= qscale;
                ndl[u] = -bc::pfma(o.x[0], dO[u].x[0], o.x[1] * dO[u].x[1]);
                lse2[u] = (f2){a.lse[ti.row * NHT + 2 * wk.hp], a.lse[ti.row * NHT + 2 * wk.hp + 1]} * kLog2e;
                char* rec = sm + kvw + beta * REC + u * 32;   // key u of quad beta
                *reinterpret_cast<bc::f4*>(rec) = (bc::f4){kr.x, kr.z, kr.y, kr.w};
                *reinterpret_cast<bc::f4*>(rec + 16) = (bc::f4){vr.x, vr.z, vr.y, vr.w};
            }
        }
        asm volatile("" ::: "memory");   // the records are written before the walk reads them
        bool ok = true;
#pragma unroll
        for (int u = 0; u < 4; ++u) ok = ok && bc::fold_ok(lse2[u]);
        const bool fold = __all(ok);
        if (fold) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const f2 e = bc::exp2_2(-lse2[u]);
                dO[u].x[0] *= e;
                dO[u].x[1] *= e;
                ndl[u] *= e;
            }
        }
#define MMNI_Q4M(M, F) \
    q4M_loop<M, F>(q, dO, lse2, ndl, dq, lcode, rq, reg, sm, kvw, dtw, lane_ok, rowk, kout, kstride, kscale)
        if (fold) {
            if (reg.masked) MMNI_Q4M(true, true);
            else MMNI_Q4M(false, true);
        } else {
            if (reg.masked) MMNI_Q4M(true, false);
            else MMNI_Q4M(false, false);
        }
#undef MMNI_Q4M
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 4; ++u) bc::store_row_nat(a.dq + (int64_t)rowk[u] * a.qs + coff, dq[u], a.scale);
        }
        asm volatile("" ::: "memory");   // the next window's records stay behind this walk's reads
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
// pass B, quad layout: lane = key quad (4 keys), the wave walks the 54 query quads; query records
// (q * scale * log2 e, dO [* 2^-lse], -delta [* 2^-lse], lse) broadcast from LDS; dk, dv in registers
// ------------------------------------------------------------------------------------
#ifndef MMNI_Q4B_UNROLL
#define MMNI_Q4B_UNROLL 6
#endif
namespace q4 {
constexpr int QREC = 192;                           // query-quad record: 4 x (q f4, dO f4, (-delta, lse) f4)
constexpr int QRB = NB * QREC;                      // 10368 B per wave
constexpr int TAB_B = WAVES * QRB;                  // bias table after the records (row bases >= 0)
constexpr int LDS_B = TAB_B + TABB;                 // 52120 B: three workgroups per CU
}  // namespace q4

template <bool MASKED, bool FOLD>
__device__ __forceinline__ void q4B_loop(const Row (&kr)[4], const Row (&vr)[4], Row (&dk)[4], Row (&dv)[4],
                                         int lcode, const int (&rk)[4], const bc::Regions& reg, const char* sm,
                                         int qrw) {
    using namespace q4;
    const char* qr = sm + qrw;
    // entry of (query quad m, row u; key row v) = code(m) - code(beta) + OFF + D(u, v); per query
    // row (zr, yr) one base, immediates (D + DMIN + x) * EB per query x
    const uint32_t lane_e = (uint32_t)((OFF - lcode - DMIN) * EB);
    for (int zr = 0; zr < 3; ++zr) {
        for (int yr = 0; yr < 3; ++yr) {
            const char* tp = sm + TAB_B + (lane_e + (uint32_t)((zr * TW + yr * TH) * EB));
            const char* qrr = qr + (zr * 3 + yr) * 6 * QREC;
#if MMNI_Q4B_UNROLL == 1
#pragma unroll 1
#elif MMNI_Q4B_UNROLL == 2
#pragma unroll 2
#elif MMNI_Q4B_UNROLL == 3
#pragma unroll 3
#else
#pragma unroll
#endif
            for (int x = 0; x < 6; ++x) {
                const char* rec = qrr + x * QREC;
                f2 bt[9];
#pragma unroll
                for (int e = 0; e < 9; ++e) bt[e] = *reinterpret_cast<const f2*>(tp + (dcode(e) + DMIN + x) * EB);
#pragma unroll
                for (int u = 0; u < 4; ++u) {       // query row u of the quad: record (q, dO, -delta, lse)
                    f2 qq[2], gg[2], nd, ls;
                    bc::ld_pair(reinterpret_cast<const f2*>(rec + u * 48), qq[0], qq[1]);
                    bc::ld_pair(reinterpret_cast<const f2*>(rec + u * 48 + 16), gg[0], gg[1]);
                    bc::ld_pair(reinterpret_cast<const f2*>(rec + u * 48 + 32), nd, ls);
                    int rq = 0;
                    if (MASKED) rq = bc::region_code(reg, zr + 3 * (u >> 1), yr + 3 * (u & 1), x);
#pragma unroll
                    for (int v = 0; v < 4; ++v) {   // the lane's key row v
                        const int e = slot(u, v);
                        f2 base = FOLD ? bt[e] : bt[e] - ls;
                        if (MASKED) base += bc::splat(rq == rk[v] ? 0.f : kMask2);
                        f2 s = bc::pfma(qq[0], kr[v].x[0], base);
                        s = bc::pfma(qq[1], kr[v].x[1], s);
                        const f2 p = bc::exp2_2(s);
                        f2 tt = bc::pfma(gg[0], vr[v].x[0], nd);
                        tt = bc::pfma(gg[1], vr[v].x[1], tt);
                        const f2 dsv = p * tt;
                        dv[v].x[0] = bc::pfma(p, gg[0], dv[v].x[0]);
                        dv[v].x[1] = bc::pfma(p, gg[1], dv[v].x[1]);
                        dk[v].x[0] = bc::pfma(dsv, qq[0], dk[v].x[0]);
                        dk[v].x[1] = bc::pfma(dsv, qq[1], dk[v].x[1]);
                    }
                }
            }
        }
    }
}

#ifndef MMNI_Q4B_WPE
#define MMNI_Q4B_WPE 2   // waves per SIMD of the quad pass B (3: 168 VGPRs, spills; measured slower)
#endif
__global__ __launch_bounds__(q4::WAVES * 64) __attribute__((amdgpu_waves_per_eu(MMNI_Q4B_WPE)))
void wattn_bwdB_q4_kernel(WAArgs a) {
    using namespace q4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    char* sm = reinterpret_cast<char*>(smem);
    const WGeom& g = a.g;
    const int NHG = a.hsplit, NHT = 2 * NHG;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const Work wk = work(NHG, wave);
    float* tab = reinterpret_cast<float*>(sm + TAB_B);
    for (int e = tid; e < TSZ * 2; e += blockDim.x) tab[e] = a.table[(e >> 1) * NHT + 2 * wk.hp + (e & 1)] * kLog2e;
    __syncthreads();
    const bool lane_ok = lane < NB;
    const int beta = lane_ok ? (int)kPermQ[lane] : 0;
    const int tb0 = base_token(beta), lcode = base_code(beta);
    const int bz = beta / 18, by = (beta / 6) % 3, bx = beta % 6;
    const int qrw = wave * QRB;
    const int coff = wk.hp * 4;
    const float qs2 = a.scale * kLog2e;
    for (int j = wk.j0;; j += wk.dj) {
        const int w = wk.xcd + 8 * j;
        if (w >= g.nwin) break;
        Row kr[4], vr[4], dk[4], dv[4];
        int rk[4] = {0, 0, 0, 0};
        int64_t row[4] = {0, 0, 0, 0};
        f2 l2[4];
        const bc::Regions reg = bc::window_regions(g, w);
        bool ok = true;
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const TokenInfo ti = token_info(g, w, tb0 + (u & 1) * 18 + (u >> 1) * 108);
                row[u] = ti.row;
                rk[u] = bc::region_code(reg, bz + 3 * (u >> 1), by + 3 * (u & 1), bx);
                l2[u] = (f2){a.lse[ti.row * NHT + 2 * wk.hp], a.lse[ti.row * NHT + 2 * wk.hp + 1]} * kLog2e;
                ok = ok && bc::fold_ok(l2[u]);
            }
        }
        // the lanes' rows are the whole window: the fold is decided per wave = per window
        const bool fold = __all(!lane_ok || ok);
        if (lane_ok) {
            char* rec = sm + qrw + beta * QREC;   // query quad beta
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                kr[u] = bc::load_row_pk(a.k + row[u] * a.ks + coff);
                vr[u] = bc::load_row_pk(a.v + row[u] * a.vs + coff);
                dk[u].x[0] = dk[u].x[1] = dv[u].x[0] = dv[u].x[1] = bc::splat(0.f);
                const float4 qv = *reinterpret_cast<const float4*>(a.q + row[u] * a.qs + coff);
                const float4 gv = *reinterpret_cast<const float4*>(a.dout + row[u] * a.os + coff);
                const float4 ov = *reinterpret_cast<const float4*>(a.o + row[u] * a.os + coff);
                const f2 e = fold ? bc::exp2_2(-l2[u]) : bc::splat(1.f);
                const float d0 = ov.x * gv.x + ov.y * gv.y, d1 = ov.z * gv.z + ov.w * gv.w;
                *reinterpret_cast<bc::f4*>(rec + u * 48) = (bc::f4){qv.x * qs2, qv.z * qs2, qv.y * qs2, qv.w * qs2};
                *reinterpret_cast<bc::f4*>(rec + u * 48 + 16) =
                    (bc::f4){gv.x * e.x, gv.z * e.y, gv.y * e.x, gv.w * e.y};
                *reinterpret_cast<bc::f4*>(rec + u * 48 + 32) = (bc::f4){-d0 * e.x, -d1 * e.y, l2[u].x, l2[u].y};
            }
        }
        asm volatile("" ::: "memory");   // the records are written before the walk reads them
        if (lane_ok) {
            if (fold) {
                if (reg.masked) q4B_loop<true, true>(kr, vr, dk, dv, lcode, rk, reg, sm, qrw);
                else q4B_loop<false, true>(kr, vr, dk, dv, lcode, rk, reg, sm, qrw);
            } else {
                if (reg.masked) q4B_loop<true, false>(kr, vr, dk, dv, lcode, rk, reg, sm, qrw);
                else q4B_loop<false, false>(kr, vr, dk, dv, lcode, rk, reg, sm, qrw);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                bc::store_row_nat(a.dv + row[u] * a.vs + coff, dv[u], 1.0f);
                bc::store_row_nat(a.dk + row[u] * a.ks + coff, dk[u], kLn2);   // staged q2 = q * scale * log2e
            }
        }
        asm volatile("" ::: "memory");   // the next window's records stay behind this walk's reads
    }
}

// ------------------------------------------------------------------------------------
// forward, quad layout: lane = query quad, key-quad records (k, v) broadcast as in pass A; online
// softmax as wattn_fwd_bc_kernel (bounded waves: no reference; others: lazy reference)
// ------------------------------------------------------------------------------------
template <bool MASKED, bool BOUNDED>
__device__ __forceinline__ void q4F_loop(const Row (&q)[4], f2 (&m)[4], f2 (&l)[4], Row (&o)[4], int lcode,
                                         const int (&rq)[4], const bc::Regions& reg, const char* sm, int kvw) {
    using namespace q4;
    const char* kv = sm + kvw;
    const char* tb = sm + TAB;
    const uint32_t lane_e = (uint32_t)((lcode + OFF - DMIN) * EB);
    f2 kk[4][2], vv[4][2], bt[9];
    auto fetch = [&](const char* rec, const char* te) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            bc::ld_pair(reinterpret_cast<const f2*>(rec + v * 32), kk[v][0], kk[v][1]);
            bc::ld_pair(reinterpret_cast<const f2*>(rec + v * 32 + 16), vv[v][0], vv[v][1]);
        }
#pragma unroll
        for (int e = 0; e < 9; ++e) bt[e] = *reinterpret_cast<const f2*>(te + (dcode(e) + DMIN) * EB);
    };
    if (BOUNDED) {
        m[0] = m[1] = m[2] = m[3] = bc::splat(0.f);
    } else {   // the reference: each row's exact maximum over key quad 0
        fetch(kv, tb + lane_e);
        int rk[4] = {0, 0, 0, 0};
        if (MASKED) {
#pragma unroll
            for (int v = 0; v < 4; ++v) rk[v] = bc::region_code(reg, 3 * (v >> 1), 3 * (v & 1), 0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            f2 mx = bc::splat(-INFINITY);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                f2 base = bt[slot(u, v)];
                if (MASKED) base += bc::splat(rk[v] == rq[u] ? 0.f : kMask2);
                f2 s = bc::pfma(q[u].x[0], kk[v][0], base);
                s = bc::pfma(q[u].x[1], kk[v][1], s);
                mx = (f2){fmaxf(mx.x, s.x), fmaxf(mx.y, s.y)};
            }
            m[u] = mx;
        }
    }
    for (int zr = 0; zr < 3; ++zr) {
        for (int yr = 0; yr < 3; ++yr) {
            const char* tp = tb + (lane_e - (uint32_t)((zr * TW + yr * TH) * EB));
            const char* kvr = kv + (zr * 3 + yr) * 6 * REC;
#pragma unroll
            for (int x = 0; x < 6; ++x) {
                fetch(kvr + x * REC, tp - x * EB);
                int rk[4] = {0, 0, 0, 0};
                if (MASKED) {
#pragma unroll
                    for (int v = 0; v < 4; ++v) rk[v] = bc::region_code(reg, zr + 3 * (v >> 1), yr + 3 * (v & 1), x);
                }
                if (BOUNDED) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
#pragma unroll
                        for (int v = 0; v < 4; ++v) {
                            f2 base = bt[slot(u, v)];
                            if (MASKED) base += bc::splat(rk[v] == rq[u] ? 0.f : kMask2);
                            f2 s = bc::pfma(q[u].x[0], kk[v][0], base);
                            s = bc::pfma(q[u].x[1], kk[v][1], s);
                            const f2 p = bc::exp2_2(s);
                            l[u] += p;
                            o[u].x[0] = bc::pfma(p, vv[v][0], o[u].x[0]);
                            o[u].x[1] = bc::pfma(p, vv[v][1], o[u].x[1]);
                        }
                    }
                    // no branch in the step: keep the compiler from hoisting the next reads (spills)
                    __builtin_amdgcn_sched_barrier(0);
                } else {
                    f2 s[4][4];
                    float smax = -INFINITY;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
#pragma unroll
                        for (int v = 0; v < 4; ++v) {
                            f2 base = bt[slot(u, v)] - m[u];
                            if (MASKED) base += bc::splat(rk[v] == rq[u] ? 0.f : kMask2);
                            f2 sv = bc::pfma(q[u].x[0], kk[v][0], base);
                            s[u][v] = bc::pfma(q[u].x[1], kk[v][1], sv);
                            smax = fmaxf(smax, fmaxf(s[u][v].x, s[u][v].y));
                        }
                    }
                    if (__any(smax > kLazy)) {   // rare: raise the reference of the rows that need it
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            f2 up = bc::splat(0.f);
#pragma unroll
                            for (int v = 0; v < 4; ++v) up = (f2){fmaxf(up.x, s[u][v].x), fmaxf(up.y, s[u][v].y)};
                            const f2 alpha = bc::exp2_2(-up);
                            l[u] *= alpha;
                            o[u].x[0] *= alpha;
                            o[u].x[1] *= alpha;
                            m[u] += up;
#pragma unroll
                            for (int v = 0; v < 4; ++v) s[u][v] -= up;
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
#pragma unroll
                        for (int v = 0; v < 4; ++v) {
                            const f2 p = bc::exp2_2(s[u][v]);
                            l[u] += p;
                            o[u].x[0] = bc::pfma(p, vv[v][0], o[u].x[0]);
                            o[u].x[1] = bc::pfma(p, vv[v][1], o[u].x[1]);
                        }
                    }
                }
            }
        }
    }
}

__global__ __launch_bounds__(q4::WAVES * 64) __attribute__((amdgpu_waves_per_eu(3)))
void wattn_fwd_q4_kernel(WAArgs a) {
    using namespace q4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    char* sm = reinterpret_cast<char*>(smem);
    const WGeom& g = a.g;
    const int NHG = a.hsplit, NHT = 2 * NHG;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const Work wk = work(NHG, wave);
    float* tab = reinterpret_cast<float*>(sm + TAB);
    float tabs = 0.f;   // this thread's entries all belong to head tid & 1 (the stride is even)
    for (int e = tid; e < TSZ * 2; e += blockDim.x) {
        const float x = a.table[(e >> 1) * NHT + 2 * wk.hp + (e & 1)] * kLog2e;
        tab[e] = x;
        tabs = fmaxf(tabs, fabsf(x));
    }
    for (int off = 2; off < 64; off <<= 1) tabs = fmaxf(tabs, __shfl_xor(tabs, off));
    float* red = reinterpret_cast<float*>(sm + LDS_F);   // [WAVES][2] max |bias| per head
    if (lane < 2) red[wave * 2 + lane] = tabs;
    __syncthreads();
    f2 tmax = bc::splat(0.f);
#pragma unroll
    for (int i = 0; i < WAVES; ++i) tmax = (f2){fmaxf(tmax.x, red[2 * i]), fmaxf(tmax.y, red[2 * i + 1])};
    const bool lane_ok = lane < NB;
    const int beta = lane_ok ? (int)kPermQ[lane] : 0;
    const int tb0 = base_token(beta), lcode = base_code(beta);
    const int bz = beta / 18, by = (beta / 6) % 3, bx = beta % 6;
    const int kvw = wave * KVB;
    const int coff = wk.hp * 4;
    const f2 qscale = bc::splat(a.scale * kLog2e);
    float vabs = 0.f;
    for (int j = wk.j0;; j += wk.dj) {
        const int w = wk.xcd + 8 * j;
        if (w >= g.nwin) break;
        Row q[4], o[4];
        f2 m[4], l[4];
        int rq[4] = {0, 0, 0, 0};
        int64_t row[4] = {0, 0, 0, 0};
        const bc::Regions reg = bc::window_regions(g, w);
        f2 kn = bc::splat(0.f);   // max |k|^2 per head over the lane's keys
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const TokenInfo ti = token_info(g, w, tb0 + (u & 1) * 18 + (u >> 1) * 108);
                row[u] = ti.row;
                rq[u] = bc::region_code(reg, bz + 3 * (u >> 1), by + 3 * (u & 1), bx);
                const float4 kr = *reinterpret_cast<const float4*>(a.k + ti.row * a.ks + coff);
                const float4 vr = *reinterpret_cast<const float4*>(a.v + ti.row * a.vs + coff);
                q[u] = bc::load_row_pk(a.q + ti.row * a.qs + coff);
                q[u].x[0] *= qscale;
                q[u].x[1] *= qscale;
                kn = (f2){fmaxf(kn.x, kr.x * kr.x + kr.y * kr.y), fmaxf(kn.y, kr.z * kr.z + kr.w * kr.w)};
                vabs = fmaxf(vabs, fmaxf(fmaxf(fabsf(vr.x), fabsf(vr.y)), fmaxf(fabsf(vr.z), fabsf(vr.w))));
                char* rec = sm + kvw + beta * REC + u * 32;
                *reinterpret_cast<bc::f4*>(rec) = (bc::f4){kr.x, kr.z, kr.y, kr.w};
                *reinterpret_cast<bc::f4*>(rec + 16) = (bc::f4){vr.x, vr.z, vr.y, vr.w};
                l[u] = bc::splat(0.f);
                o[u].x[0] = o[u].x[1] = bc::splat(0.f);
            }
        }
        asm volatile("" ::: "memory");   // the records are written before the walk reads them
        for (int off = 1; off < 64; off <<= 1)
            kn = (f2){fmaxf(kn.x, __shfl_xor(kn.x, off)), fmaxf(kn.y, __shfl_xor(kn.y, off))};
        bool rows_ok = true;
        if (lane_ok) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const f2 qn = bc::pfma(q[u].x[0], q[u].x[0], q[u].x[1] * q[u].x[1]);
                const f2 qk = qn * kn;
                rows_ok = rows_ok && __builtin_sqrtf(qk.x) + tmax.x <= kFwdBound &&
                          __builtin_sqrtf(qk.y) + tmax.y <= kFwdBound;
            }
        }
        const bool bounded = __all(rows_ok);
        if (lane_ok) {
            if (bounded) {
                if (reg.masked) q4F_loop<true, true>(q, m, l, o, lcode, rq, reg, sm, kvw);
                else q4F_loop<false, true>(q, m, l, o, lcode, rq, reg, sm, kvw);
            } else {
                if (reg.masked) q4F_loop<true, false>(q, m, l, o, lcode, rq, reg, sm, kvw);
                else q4F_loop<false, false>(q, m, l, o, lcode, rq, reg, sm, kvw);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const f2 inv = (f2){1.0f / l[u].x, 1.0f / l[u].y};
                Row r;
                r.x[0] = o[u].x[0] * inv;
                r.x[1] = o[u].x[1] * inv;
                bc::store_row_nat(a.out + row[u] * a.os + coff, r, 1.0f);
                a.lse[row[u] * NHT + 2 * wk.hp] = (m[u].x + fast_log2(l[u].x)) * kLn2;
                a.lse[row[u] * NHT + 2 * wk.hp + 1] = (m[u].y + fast_log2(l[u].y)) * kLn2;
            }
        }
        asm volatile("" ::: "memory");   // the next window's records stay behind this walk's reads
    }
    if (a.vmax != nullptr) {
        for (int off = 32; off > 0; off >>= 1) vabs = fmaxf(vabs, __shfl_xor(vabs, off));
        if (lane == 0) atomicMax(a.vmax, __float_as_uint(vabs));
    }
}

__global__ void wattn_dtable_add_kernel(const float* src, float* dtable, int n) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) dtable[e] += src[e];
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

static size_t bcA_lds() { return (size_t)bc::align4(bc::Win<6, 6, 6>::TSZ * 6) * 4 + (size_t)8 * bc::Win<6, 6, 6>::H * 8; }
static size_t bcB_lds() { return (size_t)bc::align4(bc::Win<6, 6, 6>::TSZ * 2) * 4 + (size_t)12 * bc::Win<6, 6, 6>::H * 8; }

// persistent grid: resident workgroups per CU from the LDS footprint and the register budget
// (waves_per_eu of the kernel: 2-wave workgroups, 4 SIMDs), a multiple of 8 * NHG
static int bc_blocks(size_t lds, int NHG, int waves_per_eu) {
    int per_cu = (int)((160 * 1024) / lds);
    if (per_cu > 2 * waves_per_eu) per_cu = 2 * waves_per_eu;
    if (per_cu < 1) per_cu = 1;
    int grid = kNumCU * per_cu;
    grid -= grid % (8 * NHG);
    return grid < 8 * NHG ? 8 * NHG : grid;
}

#ifndef MMNI_BWDA_Q4
#define MMNI_BWDA_Q4 1   // pass A in the quad layout (0: the row-pair kernel)
#endif

#ifndef MMNI_BWDB_Q4
#define MMNI_BWDB_Q4 1   // pass B in the quad layout
#endif
#ifndef MMNI_FWD_Q4
#define MMNI_FWD_Q4 0    // forward in the quad layout (measured 5% slower than the row-pair kernel)
#endif

// quad kernels: per_cu resident 4-wave workgroups per CU (pass A: 2 by LDS; pass B and the
// forward: 3 by registers), a multiple of 8 with every head pair served
static int q4_blocks(int per_cu, int NHG) {
    int grid = per_cu * kNumCU;
    grid -= grid % 8;
    return grid < 8 * NHG ? 8 * NHG : grid;
}

#ifndef MMNI_BWD_MERGED
#define MMNI_BWD_MERGED 1   // one merged quad kernel (dq, dk, dv, table) instead of passes A and B
#endif

static int bwdA_grid(int NHG) {
    return (MMNI_BWDA_Q4 || MMNI_BWD_MERGED) ? q4_blocks(2, NHG) : bc_blocks(bcA_lds(), NHG, 2);
}

size_t wattn_bc_workspace_bytes(const WGeom& g, int heads) {
    const int gridA = bwdA_grid(heads / 2);
    return ((size_t)gridA + 1) * g.Tsz * heads * sizeof(float);
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

static size_t bcF_lds() { return (size_t)bc::align4(bc::Win<6, 6, 6>::TSZ * 2) * 4 + (size_t)8 * bc::Win<6, 6, 6>::H * 8 + 8 * 4; }

int wattn_bc_forward(WAArgs& a, int heads, hipStream_t s) {
    const WGeom& g = a.g;
    constexpr int kTsz666 = bc::Win<6, 6, 6>::TSZ;
    MMNI_ARG_CHECK(g.wd == 6 && g.wh == 6 && g.ww == 6 && g.Tsz == kTsz666, "wattn_fwd (broadcast): compiled for 6^3 windows");
    const int NHG = heads / 2;
    a.hsplit = NHG;
    if (MMNI_FWD_Q4) {
        const size_t lds = (size_t)q4::LDS_F + 8 * sizeof(float);
        const int grid = q4_blocks(3, NHG);
        wattn_fwd_q4_kernel<<<grid, q4::WAVES * 64, lds, s>>>(a);
        return launch_status("wattn_fwd_q4");
    }
    const size_t lds = bcF_lds();
    const int grid = bc_blocks(lds, NHG, 4);
    int rc = set_lds_limit(reinterpret_cast<const void*>(&wattn_fwd_bc_kernel<6, 6, 6>), lds);
    if (rc) return rc;
    wattn_fwd_bc_kernel<6, 6, 6><<<grid, bc::kThreads, lds, s>>>(a);
    return launch_status("wattn_fwd_bc");
}

int wattn_bc_backward(WAArgs& a, int heads, float* dtable, void* workspace, hipStream_t s) {
    const WGeom& g = a.g;
    constexpr int kTsz666 = bc::Win<6, 6, 6>::TSZ;
    MMNI_ARG_CHECK(g.wd == 6 && g.wh == 6 && g.ww == 6 && g.Tsz == kTsz666, "wattn_bwd (broadcast): compiled for 6^3 windows");
    const int NHG = heads / 2;
    a.hsplit = NHG;
    const size_t ldsA = bcA_lds(), ldsB = bcB_lds();
    const int gridA = bwdA_grid(NHG), gridB = MMNI_BWDB_Q4 ? q4_blocks(MMNI_Q4B_WPE, NHG) : bc_blocks(ldsB, NHG, 3);
    const void* kA = MMNI_BWDA_Q4 ? reinterpret_cast<const void*>(&wattn_bwdA_q4_kernel)
                                  : reinterpret_cast<const void*>(&wattn_bwdA_bc_kernel<6, 6, 6>);
    const void* kB = reinterpret_cast<const void*>(&wattn_bwdB_bc_kernel<6, 6, 6>);
    int rc = set_lds_limit(kA, MMNI_BWDA_Q4 ? (size_t)q4::LDS_A : ldsA);
    if (rc) return rc;
    rc = MMNI_BWDB_Q4 ? 0 : set_lds_limit(kB, ldsB);
    if (rc) return rc;
    const int ncol = g.Tsz * heads;
    float* part = static_cast<float*>(workspace);          // [gridA][Tsz * heads]
    float* sum = part + (size_t)gridA * ncol;              // [Tsz * heads]
    if (MMNI_BWD_MERGED) {
        rc = set_lds_limit(reinterpret_cast<const void*>(&wattn_bwd_q4m_kernel), q4::LDS_A);
        if (rc) return rc;
        wattn_bwd_q4m_kernel<<<gridA, q4::WAVES * 64, q4::LDS_A, s>>>(a, part);
        rc = launch_status("wattn_bwd_q4m");
        if (rc) return rc;
    } else {
        if (MMNI_BWDA_Q4) wattn_bwdA_q4_kernel<<<gridA, q4::WAVES * 64, q4::LDS_A, s>>>(a, part);
        else wattn_bwdA_bc_kernel<6, 6, 6><<<gridA, bc::kThreads, ldsA, s>>>(a, part);
        rc = launch_status("wattn_bwdA_bc");
        if (rc) return rc;
        if (MMNI_BWDB_Q4) wattn_bwdB_q4_kernel<<<gridB, q4::WAVES * 64, q4::LDS_B, s>>>(a);
        else wattn_bwdB_bc_kernel<6, 6, 6><<<gridB, bc::kThreads, ldsB, s>>>(a);
        rc = launch_status("wattn_bwdB_bc");
        if (rc) return rc;
    }
    column_sum(part, gridA, ncol, sum, ncol, nullptr, s);
    rc = launch_status("wattn_bwd_dtable_sum");
    if (rc) return rc;
    wattn_dtable_add_kernel<<<(ncol + 255) / 256, 256, 0, s>>>(sum, dtable, ncol);
    return launch_status("wattn_bwd_dtable_add");
}

}  // namespace mmni
