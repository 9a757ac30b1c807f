// Crossmodal multi-head attention core for gfx950.
//
// Replaces the bmm -> (+causal mask) -> fp32 softmax -> dropout -> bmm section of
//   MultiheadAttention.forward   modules/multihead_attention.py:109-125
// with buffered_future_mask      modules/crossmodal_transformer.py:179-186
// (mask = -inf where key - query >= causal_diag = 1 + |Tk - Tq|).
// The in_proj / out_proj GEMMs stay on hipBLASLt through torch.
//
// Layout: time-major (T, B, E) exactly as the reference passes it, read in place — element
// (t, b, head, c) at ptr[(t*B + b)*stride + head*hd + c] — so the reference's
// .view(T, B*h, d).transpose(0,1) copies (multihead_attention.py:92-96) never happen.
//
// Contractions on the bf16 matrix cores (v_mfma_f32_16x16x32_bf16) with every fp32 operand split
// into bf16 hi + lo parts and three products hi*hi + hi*lo + lo*hi accumulated in fp32: relative
// error ~2^-16 per product, i.e. fp32-class results at 16x the f32 MFMA rate (gfx950 has no xf32).
// head_dim d is padded to HDP = 4, 8 or 16 (7 -> 8, 14 -> 16).  One wave owns 16 rows; tiles of 64
// rows of the other operand are staged in LDS as bf16 split images and consumed as 4 sub-tiles:
//   S-type  (contraction over d)   S^T = K Q^T etc.: the 3 terms are laid along the MFMA's K = 32
//           (LDS side [hi | hi | lo], register side [hi | lo | hi]); one MFMA per 16 x 16 sub-tile
//           for d <= 8, two for d = 16.
//   Z-type  (contraction over rows) O^T += V^T P^T etc.: the fp32 MFMA accumulator of the S-type
//           product is split in registers and is the B operand as it lies (its rows are the K
//           index).  d <= 8: rows 0-7 of the A image carry Zh (x [Wh | Wl]) and rows 8-15 Zl
//           (x [Wh | 0]), one MFMA per 16 rows, halves summed once at the end; d = 16: three MFMAs
//           per 32 rows.
//   forward   S^T = K Q^T, O^T += V^T P^T
//   dq        S^T, dP^T = V dO^T, dS^T, dQ^T += K^T dS^T
//   dk, dv    S = Q K^T, dP = dO V^T, dS, dV^T += dO^T P, dK^T += Q^T dS
// Online softmax in the log2 domain: each lane holds 4 keys of one query per sub-tile; the row
// max is two cross-lane shuffles per 64 keys.  Without dropout and with d < HDP the softmax
// denominator rides in the padding row of V (ones), so the MFMA forms it.  The backward folds
// -lse and -delta into the accumulator initialisation.  Causal tiles past a wave's diagonal are
// skipped.  No atomics: deterministic.
//
// Attention dropout (multihead_attention.py:123, F.dropout on the probabilities, reference default
// --attn_dropout 0.1, main.py:176): counter-based, keep(b*h, i, j) = hash(seed, (b*h)*Tq + i, j)
// < (1 - p) * 2^32, regenerated identically in the backward and by mmni_mha_dropout_mask.
#include "mmni_common.h"
#include <type_traits>

namespace mmni {

typedef float mf4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ mf4 mfma_bf(u4 a, u4 b, mf4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}

// element I/O: fp32 or bf16 storage, fp32 arithmetic
template <typename T>
__device__ __forceinline__ float ldf(const void* p, int64_t i) {
    return (float)static_cast<const T*>(p)[i];
}
template <typename T>
__device__ __forceinline__ void stf(void* p, int64_t i, float v) {
    static_cast<T*>(p)[i] = (T)v;
}
template <typename T>
constexpr int kTerms = std::is_same<T, float>::value ? 3 : 1;   // bf16 products per fp32 product

// bf16 split of fp32: hi = truncation (exact as an fp32), lo = round(x - hi)
__device__ __forceinline__ float bf_hi(float x) { return __uint_as_float(__float_as_uint(x) & 0xffff0000u); }
__device__ __forceinline__ uint32_t pk_hi(float a, float b) {   // {hi(a), hi(b)}
    return __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x07060302u);
}
__device__ __forceinline__ uint32_t pk_rn(float a, float b) {
    bf16x2 r;
    r[0] = (__bf16)a;
    r[1] = (__bf16)b;
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t pk_lo(float a, float b) { return pk_rn(a - bf_hi(a), b - bf_hi(b)); }

struct MhaArgs {
    int Tq, Tk, B, H, hd, causal;   // causal: diag (<=0 none)
    float scale;
    float scale2;                   // scale * log2(e)
    int64_t qs, ks, vs, os;
    const void* q;                  // q / k / v / o / dout / out / dq / dk / dv: fp32 or bf16 (dtype)
    const void* k;
    const void* v;
    void* out;
    float* lse;                     // (B, H, Tq) natural log
    const void* o;
    const void* dout;
    void* dq;
    void* dk;
    void* dv;
    float* delta;                   // (B, H, Tq)
    float* probs;                   // (B, Tq, Tk)
    float inv_keep;                 // 1 / (1 - p)
    uint32_t thresh;                // keep iff hash < thresh
    uint32_t seed;
    int nqt, nkt;                   // 64-row tiles of the query / key sequences
    int bf16;                       // element type of q/k/v/o/dout and of the outputs
    // bf16 split images in the workspace (mha_split_kernel), [bh][tile][...]
    const uint16_t* kx;             // K ext
    const uint16_t* kz;             // K Z
    const uint16_t* vx;             // V ext
    const uint16_t* vz;             // V Z (forward: padding row of ones)
    const uint16_t* qx;             // Q * scale * log2e ext
    const uint16_t* qz;             // Q * scale * log2e Z
    const uint16_t* gx;             // dO ext
    const uint16_t* gz;             // dO Z
};

constexpr int MT = 64;      // rows per LDS tile and per workgroup (4 waves x 16)

// LDS image geometry per padded head_dim
// TERMS = 3 (fp32 data: hi/lo split, three products) or 1 (bf16 data: one product)
template <int HDP, int TERMS = 3>
struct Geo {
    static constexpr int NX = (TERMS * HDP + 31) / 32;   // S-type MFMAs per 16 x 16 sub-tile
    // CMP: one bf16 term of d >= 8 -- the ext row holds only the d live values (16 / 32 B) instead of
    // a zero-padded K = 32 row.  Lanes past K = d read live data of their own row (8 (lg mod d/8)):
    // the register side is zero there, so those products vanish.  Each ds_read_b128 lane group then
    // covers the 16 rows once: no bank conflicts (a padded 80-B row measured 41% conflict cycles).
    static constexpr bool CMP = TERMS == 1 && HDP >= 8;
    static constexpr int XS = CMP ? HDP : 32 * NX + 8;   // ext image row stride in LDS (bf16)
    static constexpr bool RS = TERMS == 3 && HDP <= 8;   // Z image: row-split (one MFMA per 16 rows)
    // Z image row stride (bf16): 272 / 144 B; CMP: 160 B, where the 16 (row, 16-B column) pairs of
    // every ds_read_b128 lane group fall on distinct bank quads (144 B: 2-way conflicts)
    static constexpr int ZS = CMP ? 80 : (RS ? 136 : 72);
    // Z image rows (RS: hi 0-7, lo 8-15; 3 terms, d = 16: hi 0-15, lo 16-31; 1 term: 0-15)
    // CMP: d rows (HDP 8: the MFMA's rows 8-15 re-read rows 0-7; their outputs, dims >= 8, are
    // never stored)
    static constexpr int ZR = CMP ? HDP : (TERMS == 1 ? 16 : (RS ? 16 : 32));
    static constexpr int EW = CMP ? HDP : 32 * NX;   // ext image row in global (unpadded)
    static constexpr int XPAD = XS - EW;             // LDS row padding of the ext image (bf16)
    static constexpr int ZW = RS ? 128 : 64;         // Z image row in global (unpadded)
    static constexpr int XT = MT * EW;               // ext tile (bf16 elements)
    static constexpr int ZT = ZR * ZW;               // Z tile (bf16 elements)
};

// ---- dropout hash (lowbias32 mixer, two rounds keyed by row then column)
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t drop_row(uint32_t seed, int bh, int Tq, int i) {
    return mix32(seed ^ mix32((uint32_t)(bh * Tq + i) * 0x9e3779b9U + 0x632be5abU));
}
__device__ __forceinline__ bool drop_keep(uint32_t rowh, int j, uint32_t thresh) {
    return mix32(rowh + (uint32_t)j * 0x85ebca6bU) < thresh;
}

// key limit (exclusive) for query row i under the causal mask
__device__ __forceinline__ int key_end(const MhaArgs& a, int i) {
    if (a.causal <= 0) return a.Tk;
    const int e = i + a.causal;
    return e < a.Tk ? e : a.Tk;
}

// XCD-aware block coordinates: workgroups are dealt to the 8 XCDs round-robin by linear id, so
// with B*H a multiple of 8 the (tile, z) blocks of head bh are all placed on XCD bh % 8 (linear id
// L: XCD L % 8, then the blocks of one bh in order) and its operand images stay in that XCD's L2.
// Used from 32 row tiles up (T >= 2,048): at T = 4,096 it measured bwd 0.427 -> 0.367 ms (bf16,
// E = 84), 0.52 -> 0.47 ms (fp32), fwd -8%; at T = 1,728 (27 tiles) the grid's own order was
// ~10% faster (scripts/bench_mha.py, alternating A/B, r3i).  Otherwise the grid's coordinates.
struct BlockXY { int x, y, z; };
__device__ __forceinline__ BlockXY xcd_block() {
    const int nx = gridDim.x, ny = gridDim.y, nz = gridDim.z;
    if (ny % 8 != 0 || nx < 32) return {(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
    const int L = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
    const int xcd = L & 7, j = L >> 3, per = nx * nz;
    const int q = j / per, r = j - q * per;
    return {r % nx, xcd + 8 * q, r / nx};
}

// block -> row tile: alternate the two ends of the sequence, so the causal mask's long and
// short tiles interleave in dispatch order (even load per CU)
__device__ __forceinline__ int zigzag(int x, int n) { return (x & 1) ? n - 1 - (x >> 1) : (x >> 1); }

template <typename T>
__device__ __forceinline__ float load_pad(const void* base, int64_t rowoff, int c, int hd, bool ok) {
    return (ok && c < hd) ? ldf<T>(base, rowoff + c) : 0.f;
}

// ------------------------------------------------------------------------------------
// split images.  mha_split_kernel writes, once per call, each operand's 64-row tiles as bf16
// images in the workspace: EXT rows [hi | hi | lo | 0] (the S-type A operand), Z rows (the Z-type
// A operand, see Geo).  The attention kernels then stage a tile with 16-byte copies.
// ------------------------------------------------------------------------------------
struct SplitOp {
    const void* x;      // (T, B, stride) time-major, head h at column h * hd (fp32 or bf16)
    int64_t xs;         // row stride of (t, b)
    int T, ntiles;
    float mul;
    int ones;           // padding dim that reads 1.0 (-1: none)
    uint16_t* ext;      // [bh][tile][MT][EW] or null
    uint16_t* z;        // [bh][tile][ZR][ZW] or null
};
struct SplitArgs {
    SplitOp op[4];
    int nops;
    int B, H, hd;
    // delta = rowsum(dO * O) as the last z-slice (backward): o/g rows with stride os
    const void* o;
    const void* g;
    int64_t os;
    int Tq;
    float* delta;       // (B, H, Tq)
};

// grid (tiles, B * H): a block builds the 64-row tile images of one head for every operand in LDS
// (all operands' loads in flight together), adds the delta rows of the tile (backward), then
// writes the images out with coalesced 16-byte stores
template <int HDP, typename T>
__global__ __launch_bounds__(256) void mha_split_kernel(SplitArgs sa) {
    constexpr int TERMS = kTerms<T>;
    using G = Geo<HDP, TERMS>;
    constexpr int IMG = G::XT + G::ZT;
    __shared__ __attribute__((aligned(16))) uint16_t img[4 * IMG];
    const int tile = blockIdx.x, bh = blockIdx.y, tid = threadIdx.x, hd = sa.hd, H = sa.H;
    const int b = bh / H, h = bh % H;
    for (int e = tid; e < sa.nops * IMG / 8; e += 256) reinterpret_cast<u4*>(img)[e] = (u4){0u, 0u, 0u, 0u};
    constexpr int DP = HDP / 2, NB = 32 * DP;   // 2 x 2 blocks (rows r, r+1; dims d, d+1) per operand
    constexpr int IT = (4 * NB + 255) / 256;
    float x[IT][2][2];
    bool live[IT];
    int T_[IT], ones_[IT];
    float mul_[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        // NB is a multiple of 64: the operand index is wave-uniform
        const int e = tid + 256 * it, o = __builtin_amdgcn_readfirstlane(e / NB), blk = e - o * NB;
        const int rp = blk / DP, dp = blk - rp * DP;
        const int oi = o < sa.nops ? o : 0;
        const T* xp = static_cast<const T*>(sa.op[oi].x);   // fields read once, up front
        const int64_t xs = sa.op[oi].xs;
        T_[it] = sa.op[oi].T;
        ones_[it] = sa.op[oi].ones;
        mul_[it] = sa.op[oi].mul;
        live[it] = (o < sa.nops) & (tile < sa.op[oi].ntiles);
        const T* src = xp + (int64_t)b * xs + h * hd;
        const int64_t rs = (int64_t)sa.B * xs;
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
            for (int dd = 0; dd < 2; ++dd)   // unconditional in-bounds loads, issued back to back
                x[it][rr][dd] = (float)src[(int64_t)min(tile * MT + 2 * rp + rr, T_[it] - 1) * rs + min(2 * dp + dd, hd - 1)];
    }
    // consume every loaded value here, so the compiler cannot sink a load under a branch below
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
            for (int dd = 0; dd < 2; ++dd) asm volatile("" : "+v"(x[it][rr][dd]));
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = tid + 256 * it, o = __builtin_amdgcn_readfirstlane(e / NB), blk = e - o * NB;
        const int rp = blk / DP, dp = blk - rp * DP;
        (void)o;
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
            for (int dd = 0; dd < 2; ++dd) {
                const int j = tile * MT + 2 * rp + rr, c = 2 * dp + dd;
                const bool ok = live[it] & (j < T_[it]);
                const float one = (ok & (c == ones_[it])) ? 1.f : 0.f;
                x[it][rr][dd] = (ok & (c < hd)) ? x[it][rr][dd] * mul_[it] : one;
            }
    }
    float dl = 0.f;   // delta of row tid (backward)
    const int di = tile * MT + tid;
    const bool dlive = sa.delta != nullptr && tid < MT && di < sa.Tq;
    if (dlive) {   // all 2 * hd loads issued together
        const int64_t off = ((int64_t)di * sa.B + b) * sa.os + h * hd;
        float ov[HDP], gv[HDP];
#pragma unroll
        for (int c = 0; c < HDP; ++c) {
            ov[c] = ldf<T>(sa.o, off + min(c, hd - 1));
            gv[c] = c < hd ? ldf<T>(sa.g, off + min(c, hd - 1)) : 0.f;
        }
#pragma unroll
        for (int c = 0; c < HDP; ++c) dl = fmaf(ov[c], gv[c], dl);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = tid + 256 * it, o = __builtin_amdgcn_readfirstlane(e / NB), blk = e - o * NB;
        if (o >= sa.nops) continue;
        const SplitOp& op = sa.op[o];
        if (tile >= op.ntiles) continue;
        const int rp = blk / DP, dp = blk - rp * DP, r = 2 * rp, d = 2 * dp;
        uint32_t* xw = reinterpret_cast<uint32_t*>(img + o * IMG);
        uint32_t* zw = reinterpret_cast<uint32_t*>(img + o * IMG + G::XT);
        if (op.ext) {
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                const int w = ((r + rr) * G::EW + d) >> 1;
                if (TERMS == 1) {   // [x | 0]
                    xw[w] = pk_rn(x[it][rr][0], x[it][rr][1]);
                    continue;
                }
                const uint32_t hi = pk_hi(x[it][rr][0], x[it][rr][1]);
                xw[w] = hi;
                xw[w + HDP / 2] = hi;
                xw[w + HDP] = pk_lo(x[it][rr][0], x[it][rr][1]);
            }
        }
        if (op.z) {
#pragma unroll
            for (int dd = 0; dd < 2; ++dd) {
                if (TERMS == 1) {   // [d][c][lg][j], one term
                    const int j = ((r >> 4) & 1) * 4 + (r & 3);
                    const int w = ((d + dd) * G::ZW + (r >> 5) * 32 + ((r & 15) >> 2) * 8 + j) >> 1;
                    zw[w] = pk_rn(x[it][0][dd], x[it][1][dd]);
                    continue;
                }
                const uint32_t hi = pk_hi(x[it][0][dd], x[it][1][dd]), lo = pk_lo(x[it][0][dd], x[it][1][dd]);
                if (G::RS) {   // [m][st][lg][j]: m < 8 hi (j and j + 4), m >= 8 lo (j < 4)
                    const int w = ((d + dd) * G::ZW + (r >> 4) * 32 + ((r & 15) >> 2) * 8 + (r & 3)) >> 1;
                    zw[w] = hi;
                    zw[w + 2] = hi;
                    zw[w + 4 * G::ZW] = lo;   // row + 8
                } else {       // [d][c][lg][j]: hi rows 0-15, lo rows 16-31
                    const int j = ((r >> 4) & 1) * 4 + (r & 3);
                    const int w = ((d + dd) * G::ZW + (r >> 5) * 32 + ((r & 15) >> 2) * 8 + j) >> 1;
                    zw[w] = hi;
                    zw[w + 8 * G::ZW] = lo;   // row + 16
                }
            }
        }
    }
    if (dlive) sa.delta[(int64_t)bh * sa.Tq + di] = dl;
    __syncthreads();
    for (int o = 0; o < sa.nops; ++o) {
        const SplitOp& op = sa.op[o];
        if (tile >= op.ntiles) continue;
        const int64_t t = (int64_t)bh * op.ntiles + tile;
        if (op.ext) {
            u4* g = reinterpret_cast<u4*>(op.ext + t * G::XT);
            for (int e = tid; e < G::XT / 8; e += 256) g[e] = reinterpret_cast<const u4*>(img + o * IMG)[e];
        }
        if (op.z) {
            u4* g = reinterpret_cast<u4*>(op.z + t * G::ZT);
            for (int e = tid; e < G::ZT / 8; e += 256) g[e] = reinterpret_cast<const u4*>(img + o * IMG + G::XT)[e];
        }
    }
}

// copy one tile image (global rows of W bf16) into LDS (rows of W + PAD bf16), in two halves so
// the next tile's loads are in flight during the current tile's MFMAs
template <int ROWS, int W, int PAD = 8, int NT = 256>
struct TileCopy {
    static constexpr int CPR = W / 8;           // 16-byte chunks per row
    static constexpr int N = ROWS * CPR;
    static constexpr int IT = (N + NT - 1) / NT;
    u4 r[IT];
    __device__ __forceinline__ void load(const uint16_t* g, int tid) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int e = tid + NT * it;
            if (N % NT == 0 || e < N) r[it] = *reinterpret_cast<const u4*>(g + e * 8);
        }
    }
    __device__ __forceinline__ void store(uint16_t* l, int tid) const {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int e = tid + NT * it;
            if (N % NT == 0 || e < N) {
                const int row = e / CPR, c = e - row * CPR;
                *reinterpret_cast<u4*>(l + row * (W + PAD) + c * 8) = r[it];
            }
        }
    }
};


// register-side ext vector [hi | lo | hi | 0] of this lane's row (v = the row, HDP floats)
template <int HDP, int TERMS>
__device__ __forceinline__ void build_y(const float (&v)[HDP], int lg, u4 (&y)[Geo<HDP, TERMS>::NX]) {
#pragma unroll
    for (int c = 0; c < Geo<HDP, TERMS>::NX; ++c)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int e = 32 * c + 8 * lg + 2 * jj;
            const int seg = e / HDP, d = e - seg * HDP;
            float x0 = 0.f, x1 = 0.f;
#pragma unroll
            for (int t = 0; t < HDP; ++t) {
                x0 = t == d ? v[t] : x0;
                x1 = t == d + 1 ? v[t] : x1;
            }
            if (TERMS == 1) y[c][jj] = seg == 0 ? pk_rn(x0, x1) : 0u;
            else y[c][jj] = (seg == 0 || seg == 2) ? pk_hi(x0, x1) : (seg == 1 ? pk_lo(x0, x1) : 0u);
        }
}

// S-type: acc += X[16 st + (lane & 15)][:] . Y[:]  over the 3-term ext dimension
template <int HDP, int TERMS>
__device__ __forceinline__ int xcol(int c, int lg) {
    using G = Geo<HDP, TERMS>;
    return G::CMP ? 8 * (lg % (HDP / 8)) : 32 * c + 8 * lg;
}
template <int HDP, int TERMS>
__device__ __forceinline__ mf4 sprod(const uint16_t* xe, int st, const u4 (&y)[Geo<HDP, TERMS>::NX], mf4 acc,
                                     int ln, int lg) {
    using G = Geo<HDP, TERMS>;
#pragma unroll
    for (int c = 0; c < G::NX; ++c)
        acc = mfma_bf(*reinterpret_cast<const u4*>(xe + (16 * st + ln) * G::XS + xcol<HDP, TERMS>(c, lg)), y[c], acc);
    return acc;
}

// Z-type: acc(d x cols) += Z^T(d x 64 rows) . W(64 rows x cols), W in accumulator layout
template <int HDP, int TERMS>
__device__ __forceinline__ mf4 zprod(const uint16_t* z, const mf4 (&w)[4], mf4 acc, int ln, int lg) {
    using G = Geo<HDP, TERMS>;
    if constexpr (TERMS == 1) {   // one MFMA per 32 rows, W rounded to bf16
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const mf4 &wa = w[2 * c], &wb = w[2 * c + 1];
            const u4 B = {pk_rn(wa[0], wa[1]), pk_rn(wa[2], wa[3]), pk_rn(wb[0], wb[1]), pk_rn(wb[2], wb[3])};
            acc = mfma_bf(*reinterpret_cast<const u4*>(z + (ln & (G::ZR - 1)) * G::ZS + c * 32 + lg * 8), B, acc);
        }
    } else if constexpr (G::RS) {
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const u4 A = *reinterpret_cast<const u4*>(z + ln * G::ZS + st * 32 + lg * 8);
            const u4 B = {pk_hi(w[st][0], w[st][1]), pk_hi(w[st][2], w[st][3]), pk_lo(w[st][0], w[st][1]),
                          pk_lo(w[st][2], w[st][3])};
            acc = mfma_bf(A, B, acc);
        }
    } else {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const mf4 &wa = w[2 * c], &wb = w[2 * c + 1];
            const u4 Bh = {pk_hi(wa[0], wa[1]), pk_hi(wa[2], wa[3]), pk_hi(wb[0], wb[1]), pk_hi(wb[2], wb[3])};
            const u4 Bl = {pk_lo(wa[0], wa[1]), pk_lo(wa[2], wa[3]), pk_lo(wb[0], wb[1]), pk_lo(wb[2], wb[3])};
            const u4 Ah = *reinterpret_cast<const u4*>(z + ln * G::ZS + c * 32 + lg * 8);
            const u4 Al = *reinterpret_cast<const u4*>(z + (16 + ln) * G::ZS + c * 32 + lg * 8);
            acc = mfma_bf(Ah, Bh, acc);
            acc = mfma_bf(Ah, Bl, acc);
            acc = mfma_bf(Al, Bh, acc);
        }
    }
    return acc;
}

// the Z-type result: row-split halves summed (rows d = 4 (lg & 1) + i then), else rows d = 4 lg + i
template <int HDP, int TERMS>
__device__ __forceinline__ mf4 zfinish(mf4 acc) {
    if constexpr (Geo<HDP, TERMS>::RS) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] += __shfl_xor(acc[i], 32);
    }
    return acc;
}
template <int HDP, int TERMS>
__device__ __forceinline__ bool zrow_owner(int lg) { return Geo<HDP, TERMS>::RS ? lg < 2 : true; }

// S^T tile of a query-row wave (lane: keys k0 + 16 st + 4 lg + i, query qi): -inf past Tk and
// under the causal mask (selects, no branches)
__device__ __forceinline__ void mask_keys(mf4 (&s)[4], int k0, int qi, int lg, const MhaArgs& a) {
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = k0 + 16 * st + 4 * lg + i;
            const bool mk = (j >= a.Tk) | ((a.causal > 0) & (j - qi >= a.causal));
            s[st][i] = mk ? -INFINITY : s[st][i];
        }
}

// LDS stages: NBUF = 2 (one barrier per tile, the next tile copied in while this one computes)
// when a stage fits 20 KB, else 1 (two barriers per tile; keeps >= 4 blocks per CU)
template <int BYTES>
struct Stages {
    static constexpr int N = BYTES <= 20 * 1024 ? 2 : 1;
};

// the tile loop shared by the three kernels: load(t) fills registers from the images of tile t,
// store(buf) writes them to LDS stage buf, body(t, buf) computes on stage buf
template <int NBUF, typename Load, typename Store, typename Body>
__device__ __forceinline__ void tile_loop(int tb, int te, Load&& load, Store&& store, Body&& body) {
    if (tb >= te) return;
    load(tb);
    if (NBUF == 2) {
        store(0);
        if (tb + 1 < te) load(tb + 1);
        __syncthreads();
    }
    for (int t = tb; t < te; ++t) {
        const int buf = NBUF == 2 ? (t - tb) & 1 : 0;
        if (NBUF == 1) {
            if (t > tb) __syncthreads();
            store(0);
            __syncthreads();
            if (t + 1 < te) load(t + 1);
        }
        body(t, buf);
        if (NBUF == 2) {
            if (t + 1 < te) {
                store(buf ^ 1);
                if (t + 2 < te) load(t + 2);
            }
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
// Online softmax with a lazy reference (as the window-attention forward): tile 0 sets each row's
// reference m to its exact maximum; later tiles start the score accumulator at -m, so p = 2^acc
// needs no subtract, and m moves (with the rescale of o and l) only when some score of the wave
// exceeds it by more than kMhaLazy.  So p <= 2^kMhaLazy: no overflow in l, o or the bf16 P.
constexpr float kMhaLazy = 8.0f;

template <int HDP, bool DROP, typename T, bool ONES>
__global__ __launch_bounds__(256) void mha_fwd_mfma_kernel(MhaArgs a) {
    constexpr int TERMS = kTerms<T>;
    using G = Geo<HDP, TERMS>;
    constexpr int SK = MT * G::XS, SV = G::ZR * G::ZS, STAGE = SK + SV;   // K ext + V Z
    constexpr int NBUF = Stages<STAGE * 2>::N;
    __shared__ __attribute__((aligned(16))) uint16_t lds[NBUF * STAGE];
    const BlockXY blk = xcd_block();
    const int bh = blk.y, b = bh / a.H, h = bh % a.H;
    const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, ln = l & 15, lg = l >> 4;
    const int bx = a.causal > 0 ? zigzag(blk.x, a.nqt) : blk.x;
    const int q0 = bx * MT + wave * 16;
    const int qi = q0 + ln;
    const bool qok = qi < a.Tq;
    u4 qy[G::NX];
    {
        float qv[HDP];
        const int64_t rq = ((int64_t)qi * a.B + b) * a.qs + h * a.hd;
#pragma unroll
        for (int d = 0; d < HDP; ++d) qv[d] = load_pad<T>(a.q, rq, d, a.hd, qok) * a.scale2;
        build_y<HDP, TERMS>(qv, lg, qy);
    }
    // ONES: the denominator rides as V's padding row of ones (the host sets it when !DROP && hd < HDP)
    const uint32_t rowh = DROP ? drop_row(a.seed, bh, a.Tq, qi) : 0u;
    const uint16_t* kxg = a.kx + (int64_t)bh * a.nkt * G::XT;
    const uint16_t* vzg = a.vz + (int64_t)bh * a.nkt * G::ZT;
    TileCopy<MT, G::EW, G::XPAD> ck;
    TileCopy<G::ZR, G::ZW, G::ZS - G::ZW> cv;
    mf4 o = {0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lsum = 0.f;
    const int kend_blk = key_end(a, min(a.Tq - 1, bx * MT + MT - 1));
    const int kend_w = q0 < a.Tq ? key_end(a, min(a.Tq - 1, q0 + 15)) : 0;
    tile_loop<NBUF>(
        0, (kend_blk + MT - 1) / MT,
        [&](int t) {
            ck.load(kxg + (int64_t)t * G::XT, tid);
            cv.load(vzg + (int64_t)t * G::ZT, tid);
        },
        [&](int buf) {
            ck.store(lds + buf * STAGE, tid);
            cv.store(lds + buf * STAGE + SK, tid);
        },
        [&](int t, int buf) {
            const int k0 = t * MT;
            if (k0 >= kend_w) return;   // wave-uniform: every key of the tile is masked for this wave
            const uint16_t* kx = lds + buf * STAGE;
            const uint16_t* vz = kx + SK;
            // tile 0 is every live wave's first tile (key 0 is visible to every row)
            const float init = t == 0 ? 0.f : -m;
            mf4 s[4];
#pragma unroll
            for (int st = 0; st < 4; ++st) s[st] = sprod<HDP, TERMS>(kx, st, qy, (mf4){init, init, init, init}, ln, lg);
            // lane: s[st][i] = S^T[key k0 + 16 st + 4 lg + i][query qi] - m (log2 domain)
            const bool edge = (k0 + MT > a.Tk) || (a.causal > 0 && k0 + MT > q0 + a.causal);
            if (edge) mask_keys(s, k0, qi, lg, a);
            float mx = -INFINITY;
#pragma unroll
            for (int st = 0; st < 4; ++st)
#pragma unroll
                for (int i = 0; i < 4; ++i) mx = fmaxf(mx, s[st][i]);
            if (t == 0 || __any(mx > kMhaLazy)) {   // wave-uniform: set or raise the reference
                mx = fmaxf(mx, __shfl_xor(mx, 16));
                mx = fmaxf(mx, __shfl_xor(mx, 32));
                // first tile: the row maximum (0 if no key is visible); later: raise by mx if positive
                const float d = t == 0 ? (mx == -INFINITY ? 0.f : mx) : fmaxf(mx, 0.f);
                if (t == 0) {
                    m = d;
                } else {
                    m += d;
                    const float alpha = fast_exp2(-d);
                    o *= alpha;
                    if (!ONES) lsum *= alpha;
                }
#pragma unroll
                for (int st = 0; st < 4; ++st)
#pragma unroll
                    for (int i = 0; i < 4; ++i) s[st][i] -= d;
            }
#pragma unroll
            for (int st = 0; st < 4; ++st) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float p = fast_exp2(s[st][i]);
                    float pv = p;
                    if (!ONES) lsum += p;
                    if (DROP) pv = drop_keep(rowh, k0 + 16 * st + 4 * lg + i, a.thresh) ? p * a.inv_keep : 0.f;
                    s[st][i] = pv;
                }
            }
            o = zprod<HDP, TERMS>(vz, s, o, ln, lg);
        });
    o = zfinish<HDP, TERMS>(o);
    if (ONES) {
        const int hd = a.hd, src = ((hd >> 2) << 4) + ln, i = hd & 3;
        const float t = i == 0 ? o[0] : (i == 1 ? o[1] : (i == 2 ? o[2] : o[3]));
        lsum = __shfl(t, src);
    } else {
        lsum += __shfl_xor(lsum, 16);
        lsum += __shfl_xor(lsum, 32);
    }
    if (qok) {
        const float inv = 1.0f / lsum;
        const int64_t orow = ((int64_t)qi * a.B + b) * a.os + h * a.hd;
        if (zrow_owner<HDP, TERMS>(lg)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = 4 * (G::RS ? (lg & 1) : lg) + i;
                if (d < a.hd) stf<T>(a.out, orow + d, o[i] * inv);
            }
        }
        if (lg == 0) a.lse[(int64_t)bh * a.Tq + qi] = (m + fast_log2(lsum)) * kLn2;
    }
}

// ------------------------------------------------------------------------------------
// dq: wave = 16 queries, loops over key tiles
// ------------------------------------------------------------------------------------
template <int HDP, int TERMS>
struct DqLds {
    using G = Geo<HDP, TERMS>;
    static constexpr int SX = MT * G::XS, SZ = G::ZR * G::ZS, STAGE = 2 * SX + SZ;   // K ext, V ext, K Z
    static constexpr int NBUF = Stages<STAGE * 2>::N;
    static constexpr int BYTES = NBUF * STAGE * 2;
};
// Row groups per wave in the backward: with one bf16 term (CMP) and head_dim <= 8 a wave takes
// RG = 2 groups of 16 rows (two-wave workgroups of 64 rows), so each tile's LDS operands, copy and
// barrier serve twice the MFMA and softmax work (T=4096 E84: 0.322 -> 0.312-0.318 ms; at head_dim
// 16 the halved wave count measured slower, 0.361 -> 0.377 ms, profiles/r3t_mha_ab.txt).
template <int HDP, int TERMS>
struct BwdRG {
    static constexpr int RG = (Geo<HDP, TERMS>::CMP && HDP == 8) ? 2 : 1;
    static constexpr int NT = 256 / RG;   // threads per workgroup
};
template <int HDP, bool DROP, typename T>
__device__ __forceinline__ void mha_dq_body(const MhaArgs& a, uint16_t* lds, int bx, int bh) {
    constexpr int TERMS = kTerms<T>;
    using G = Geo<HDP, TERMS>;
    using L = DqLds<HDP, TERMS>;
    constexpr int SX = L::SX, SZ = L::SZ, STAGE = L::STAGE;
    constexpr int NBUF = L::NBUF;
    constexpr int RG = BwdRG<HDP, TERMS>::RG, NT = BwdRG<HDP, TERMS>::NT;
    (void)SZ;
    const int b = bh / a.H, h = bh % a.H;
    const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, ln = l & 15, lg = l >> 4;
    const int q0 = bx * MT + wave * 16 * RG;   // group g: rows q0 + 16 g + ln
    int qi[RG];
    bool qok[RG];
    int64_t rq[RG];
    u4 qy[RG][G::NX], gy[RG][G::NX];
    float dl[RG];
    uint32_t rowh[RG];
    mf4 sinit[RG], dinit[RG], dq[RG];
#pragma unroll
    for (int g = 0; g < RG; ++g) {
        qi[g] = q0 + 16 * g + ln;
        qok[g] = qi[g] < a.Tq;
        rq[g] = ((int64_t)qi[g] * a.B + b) * a.qs + h * a.hd;
        const int64_t ro = ((int64_t)qi[g] * a.B + b) * a.os + h * a.hd;
        float qv[HDP], gv[HDP];
#pragma unroll
        for (int d = 0; d < HDP; ++d) {
            qv[d] = load_pad<T>(a.q, rq[g], d, a.hd, qok[g]) * a.scale2;
            gv[d] = load_pad<T>(a.dout, ro, d, a.hd, qok[g]);
        }
        build_y<HDP, TERMS>(qv, lg, qy[g]);
        build_y<HDP, TERMS>(gv, lg, gy[g]);
        const float lse2 = qok[g] ? a.lse[(int64_t)bh * a.Tq + qi[g]] * kLog2e : INFINITY;
        dl[g] = qok[g] ? a.delta[(int64_t)bh * a.Tq + qi[g]] : 0.f;
        rowh[g] = DROP ? drop_row(a.seed, bh, a.Tq, qi[g]) : 0u;
        sinit[g] = (mf4){-lse2, -lse2, -lse2, -lse2};
        const float di = DROP ? 0.f : -dl[g];
        dinit[g] = (mf4){di, di, di, di};
        dq[g] = (mf4){0.f, 0.f, 0.f, 0.f};
    }
    const uint16_t* kxg = a.kx + (int64_t)bh * a.nkt * G::XT;
    const uint16_t* vxg = a.vx + (int64_t)bh * a.nkt * G::XT;
    const uint16_t* kzg = a.kz + (int64_t)bh * a.nkt * G::ZT;
    TileCopy<MT, G::EW, G::XPAD, NT> ck, cv;
    TileCopy<G::ZR, G::ZW, G::ZS - G::ZW, NT> cz;
    const int kend_blk = key_end(a, min(a.Tq - 1, bx * MT + MT - 1));
    const int kend_w = q0 < a.Tq ? key_end(a, min(a.Tq - 1, q0 + 16 * RG - 1)) : 0;
    tile_loop<NBUF>(
        0, (kend_blk + MT - 1) / MT,
        [&](int t) {
            ck.load(kxg + (int64_t)t * G::XT, tid);
            cv.load(vxg + (int64_t)t * G::XT, tid);
            cz.load(kzg + (int64_t)t * G::ZT, tid);
        },
        [&](int buf) {
            uint16_t* st = lds + buf * STAGE;
            ck.store(st, tid);
            cv.store(st + SX, tid);
            cz.store(st + 2 * SX, tid);
        },
        [&](int t, int buf) {
            const int k0 = t * MT;
            if (k0 >= kend_w) return;
            const uint16_t* kx = lds + buf * STAGE;
            const uint16_t* vx = kx + SX;
            const uint16_t* kz = kx + 2 * SX;
#pragma unroll
            for (int g = 0; g < RG; ++g) {
                const int qg = q0 + 16 * g;
                if (RG > 1 && k0 >= key_end(a, min(a.Tq - 1, qg + 15))) continue;   // wave-uniform
                mf4 s[4], dp[4];
#pragma unroll
                for (int st = 0; st < 4; ++st) {
                    s[st] = sprod<HDP, TERMS>(kx, st, qy[g], sinit[g], ln, lg);    // S^T - lse2
                    dp[st] = sprod<HDP, TERMS>(vx, st, gy[g], dinit[g], ln, lg);   // dP^T (- delta)
                }
                const bool edge = (k0 + MT > a.Tk) || (a.causal > 0 && k0 + MT > qg + a.causal);
                if (edge) mask_keys(s, k0, qi[g], lg, a);
#pragma unroll
                for (int st = 0; st < 4; ++st) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int j = k0 + 16 * st + 4 * lg + i;
                        const float p = fast_exp2(s[st][i]);
                        float gg = dp[st][i];
                        if (DROP) gg = (drop_keep(rowh[g], j, a.thresh) ? gg * a.inv_keep : 0.f) - dl[g];
                        s[st][i] = p * gg;   // dS^T
                    }
                }
                dq[g] = zprod<HDP, TERMS>(kz, s, dq[g], ln, lg);   // dQ^T += K^T dS^T
            }
        });
#pragma unroll
    for (int g = 0; g < RG; ++g) {
        const mf4 dqf = zfinish<HDP, TERMS>(dq[g]);
        if (qok[g] && zrow_owner<HDP, TERMS>(lg)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = 4 * (G::RS ? (lg & 1) : lg) + i;
                if (d < a.hd) stf<T>(a.dq, rq[g] + d, dqf[i] * a.scale);
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// dk, dv: wave = 16 keys, loops over query tiles
// ------------------------------------------------------------------------------------
template <int HDP, int TERMS>
struct DkvLds {
    using G = Geo<HDP, TERMS>;
    static constexpr int SX = MT * G::XS, SZ = G::ZR * G::ZS;
    static constexpr int STAGE = 2 * SX + 2 * SZ + 4 * MT;   // Q ext, dO ext, Q Z, dO Z, -lse2 and -delta (fp32)
    static constexpr int NBUF = Stages<STAGE * 2>::N;
    static constexpr int BYTES = NBUF * STAGE * 2;
};
template <int HDP, bool DROP, typename T>
__device__ __forceinline__ void mha_dkv_body(const MhaArgs& a, uint16_t* lds, int bx, int bh) {
    constexpr int TERMS = kTerms<T>;
    using G = Geo<HDP, TERMS>;
    using L = DkvLds<HDP, TERMS>;
    constexpr int SX = L::SX, SZ = L::SZ, STAGE = L::STAGE;
    constexpr int NBUF = L::NBUF;
    constexpr int RG = BwdRG<HDP, TERMS>::RG, NT = BwdRG<HDP, TERMS>::NT;
    const int b = bh / a.H, h = bh % a.H;
    const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, ln = l & 15, lg = l >> 4;
    const int j0 = bx * MT + wave * 16 * RG;   // group g: keys j0 + 16 g + ln
    int kj[RG];
    bool kok[RG];
    int64_t rk[RG], rv[RG];
    u4 ky[RG][G::NX], vy[RG][G::NX];
    mf4 dk[RG], dv[RG];
#pragma unroll
    for (int g = 0; g < RG; ++g) {
        kj[g] = j0 + 16 * g + ln;
        kok[g] = kj[g] < a.Tk;
        rk[g] = ((int64_t)kj[g] * a.B + b) * a.ks + h * a.hd;
        rv[g] = ((int64_t)kj[g] * a.B + b) * a.vs + h * a.hd;
        float kv[HDP], vv[HDP];
#pragma unroll
        for (int d = 0; d < HDP; ++d) {
            kv[d] = load_pad<T>(a.k, rk[g], d, a.hd, kok[g]);
            vv[d] = load_pad<T>(a.v, rv[g], d, a.hd, kok[g]);
        }
        build_y<HDP, TERMS>(kv, lg, ky[g]);
        build_y<HDP, TERMS>(vv, lg, vy[g]);
        dk[g] = dv[g] = (mf4){0.f, 0.f, 0.f, 0.f};
    }
    const uint16_t* qxg = a.qx + (int64_t)bh * a.nqt * G::XT;
    const uint16_t* gxg = a.gx + (int64_t)bh * a.nqt * G::XT;
    const uint16_t* qzg = a.qz + (int64_t)bh * a.nqt * G::ZT;
    const uint16_t* gzg = a.gz + (int64_t)bh * a.nqt * G::ZT;
    TileCopy<MT, G::EW, G::XPAD, NT> cq, cg;
    TileCopy<G::ZR, G::ZW, G::ZS - G::ZW, NT> czq, czg;
    float pl = 0.f, pd_ = 0.f;   // the tile's -lse2 / -delta (threads < MT)
    // first query that can see the block's first key: j - i < diag  <=>  i > j - diag
    int i_begin = 0;
    if (a.causal > 0) i_begin = max(0, bx * MT - a.causal + 1);
    const int ib_w = a.causal > 0 ? max(0, j0 - a.causal + 1) : 0;   // this wave's first visible query
    tile_loop<NBUF>(
        i_begin / MT, a.nqt,
        [&](int t) {
            cq.load(qxg + (int64_t)t * G::XT, tid);
            cg.load(gxg + (int64_t)t * G::XT, tid);
            czq.load(qzg + (int64_t)t * G::ZT, tid);
            czg.load(gzg + (int64_t)t * G::ZT, tid);
            if (tid < MT) {
                const int i = t * MT + tid;
                pl = i < a.Tq ? -a.lse[(int64_t)bh * a.Tq + i] * kLog2e : -INFINITY;
                pd_ = i < a.Tq ? -a.delta[(int64_t)bh * a.Tq + i] : 0.f;
            }
        },
        [&](int buf) {
            uint16_t* st = lds + buf * STAGE;
            cq.store(st, tid);
            cg.store(st + SX, tid);
            czq.store(st + 2 * SX, tid);
            czg.store(st + 2 * SX + SZ, tid);
            float* f = reinterpret_cast<float*>(st + 2 * SX + 2 * SZ);
            if (tid < MT) {
                f[tid] = pl;
                f[MT + tid] = pd_;
            }
        },
        [&](int t, int buf) {
            const int i0 = t * MT;
            if (i0 + MT <= ib_w || j0 >= a.Tk) return;   // wave-uniform: nothing visible
            const uint16_t* qx = lds + buf * STAGE;
            const uint16_t* gx = qx + SX;
            const uint16_t* qz = qx + 2 * SX;
            const uint16_t* gz = qz + SZ;
            const float* ls_ = reinterpret_cast<const float*>(qx + 2 * SX + 2 * SZ);
            const float* ds_ = ls_ + MT;
            mf4 li[4], di[4];   // the rows' -lse2 / -delta, shared by the groups
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const float2 l01 = *reinterpret_cast<const float2*>(ls_ + 16 * st + 4 * lg);
                const float2 l23 = *reinterpret_cast<const float2*>(ls_ + 16 * st + 4 * lg + 2);
                li[st] = (mf4){l01.x, l01.y, l23.x, l23.y};
                di[st] = (mf4){0.f, 0.f, 0.f, 0.f};
                if (!DROP) {
                    const float2 d01 = *reinterpret_cast<const float2*>(ds_ + 16 * st + 4 * lg);
                    const float2 d23 = *reinterpret_cast<const float2*>(ds_ + 16 * st + 4 * lg + 2);
                    di[st] = (mf4){d01.x, d01.y, d23.x, d23.y};
                }
            }
#pragma unroll
            for (int g = 0; g < RG; ++g) {
                const int jg = j0 + 16 * g;
                if (RG > 1 && (jg >= a.Tk || (a.causal > 0 && i0 + MT <= jg - a.causal + 1))) continue;   // wave-uniform
                mf4 s[4], dp[4];
#pragma unroll
                for (int st = 0; st < 4; ++st) {
                    s[st] = sprod<HDP, TERMS>(qx, st, ky[g], li[st], ln, lg);    // S - lse2
                    dp[st] = sprod<HDP, TERMS>(gx, st, vy[g], di[st], ln, lg);   // dP (- delta)
                }
                // lane: s[st][i] = S[query i0 + 16 st + 4 lg + i][key kj]
                const bool edge = (i0 + MT > a.Tq) || !kok[g] || (a.causal > 0 && i0 < jg + 16 - a.causal + 1);
                if (edge) {
#pragma unroll
                    for (int st = 0; st < 4; ++st)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int qi = i0 + 16 * st + 4 * lg + i;
                            const bool mk = (qi >= a.Tq) | !kok[g] | ((a.causal > 0) & (kj[g] - qi >= a.causal));
                            s[st][i] = mk ? -INFINITY : s[st][i];
                        }
                }
                mf4 pd[4];
#pragma unroll
                for (int st = 0; st < 4; ++st) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = 16 * st + 4 * lg + i, qi = i0 + r;
                        const float p = fast_exp2(s[st][i]);
                        float gg = dp[st][i], pv = p;
                        if (DROP) {
                            const bool kp = drop_keep(drop_row(a.seed, bh, a.Tq, qi), kj[g], a.thresh);
                            gg = (kp ? gg * a.inv_keep : 0.f) + ds_[r];
                            pv = kp ? p * a.inv_keep : 0.f;
                        }
                        pd[st][i] = pv;
                        s[st][i] = p * gg;   // dS
                    }
                }
                dv[g] = zprod<HDP, TERMS>(gz, pd, dv[g], ln, lg);   // dV^T += dO^T Pd
                dk[g] = zprod<HDP, TERMS>(qz, s, dk[g], ln, lg);    // dK^T += Q2^T dS
            }
        });
#pragma unroll
    for (int g = 0; g < RG; ++g) {
        const mf4 dkf = zfinish<HDP, TERMS>(dk[g]);
        const mf4 dvf = zfinish<HDP, TERMS>(dv[g]);
        if (kok[g] && zrow_owner<HDP, TERMS>(lg)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = 4 * (G::RS ? (lg & 1) : lg) + i;
                if (d < a.hd) {
                    stf<T>(a.dk, rk[g] + d, dkf[i] * kLn2);   // staged q2 = q * scale * log2e
                    stf<T>(a.dv, rv[g] + d, dvf[i]);
                }
            }
        }
    }
}

// the backward's two halves in one launch: z = 0 dq blocks (query tiles), z = 1 dk/dv blocks (key
// tiles); dq's causal tail overlaps the first dk/dv blocks
template <int HDP, bool DROP, typename T>
__global__ __launch_bounds__(256) void mha_bwd_mfma_kernel(MhaArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t dyn_lds[];
    const BlockXY blk = xcd_block();
    if (blk.z == 0) {
        if (blk.x >= a.nqt) return;
        mha_dq_body<HDP, DROP, T>(a, dyn_lds, a.causal > 0 ? zigzag(blk.x, a.nqt) : blk.x, blk.y);
    } else {
        if (blk.x >= a.nkt) return;
        mha_dkv_body<HDP, DROP, T>(a, dyn_lds, a.causal > 0 ? zigzag(blk.x, a.nkt) : blk.x, blk.y);
    }
}

// head-averaged (dropped) probabilities: probs[b, i, j] = mean_h keep * softmax_j(...) / (1 - p)
template <bool DROP, typename T>
__global__ __launch_bounds__(256) void mha_probs_kernel(MhaArgs a) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over (b, i, j)
    if (e >= (int64_t)a.B * a.Tq * a.Tk) return;
    const int j = (int)(e % a.Tk);
    const int64_t bi = e / a.Tk;
    const int i = (int)(bi % a.Tq), b = (int)(bi / a.Tq);
    float sum = 0.f;
    const bool vis = a.causal <= 0 || j - i < a.causal;
    if (vis) {
        for (int h = 0; h < a.H; ++h) {
            const int64_t qo = ((int64_t)i * a.B + b) * a.qs + h * a.hd;
            const int64_t ko = ((int64_t)j * a.B + b) * a.ks + h * a.hd;
            float s = 0.f;
            for (int c = 0; c < a.hd; ++c) s = fmaf(ldf<T>(a.q, qo + c), ldf<T>(a.k, ko + c), s);
            float p = fast_exp2(s * a.scale2 - a.lse[((int64_t)b * a.H + h) * a.Tq + i] * kLog2e);
            if (DROP) p = drop_keep(drop_row(a.seed, b * a.H + h, a.Tq, i), j, a.thresh) ? p * a.inv_keep : 0.f;
            sum += p;
        }
    }
    a.probs[e] = sum / (float)a.H;
}

// the dropout multipliers (0 or 1 / (1 - p)) of every (b, h, i, j), for tests
__global__ __launch_bounds__(256) void mha_dropout_mask_kernel(MhaArgs a, float* mask) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over (bh, i, j)
    if (e >= (int64_t)a.B * a.H * a.Tq * a.Tk) return;
    const int j = (int)(e % a.Tk);
    const int64_t r = e / a.Tk;
    const int i = (int)(r % a.Tq), bh = (int)(r / a.Tq);
    mask[e] = drop_keep(drop_row(a.seed, bh, a.Tq, i), j, a.thresh) ? a.inv_keep : 0.f;
}

static int mha_fill(const mmni_mha_desc* d, MhaArgs& a) {
    MMNI_ARG_CHECK(d != nullptr, "mha: null descriptor");
    MMNI_ARG_CHECK(d->Tq > 0 && d->Tk > 0 && d->B > 0 && d->heads > 0 && d->head_dim > 0, "mha: bad sizes");
    if (d->head_dim > 16) {
        set_error("mha: unsupported head_dim %d (supported 1..16)", d->head_dim);
        return -2;
    }
    const int E = d->heads * d->head_dim;
    MMNI_ARG_CHECK(d->q_stride >= E && d->k_stride >= E && d->v_stride >= E && d->o_stride >= E,
                   "mha: strides must be >= heads*head_dim");
    MMNI_ARG_CHECK((int64_t)d->B * d->heads <= 65535, "mha: B*heads exceeds the grid y limit");
    MMNI_ARG_CHECK((int64_t)d->B * d->heads * d->Tq < (1ll << 31), "mha: too many rows");
    MMNI_ARG_CHECK(d->dropout >= 0.f && d->dropout < 1.f, "mha: dropout must be in [0, 1)");
    MMNI_ARG_CHECK(d->dtype == 0 || d->dtype == 1, "mha: dtype must be 0 (fp32) or 1 (bf16)");
    a.Tq = d->Tq; a.Tk = d->Tk; a.B = d->B; a.H = d->heads; a.hd = d->head_dim; a.causal = d->causal_diag;
    a.scale = d->scale;
    a.scale2 = d->scale * kLog2e;
    a.qs = d->q_stride; a.ks = d->k_stride; a.vs = d->v_stride; a.os = d->o_stride;
    const double keep = 1.0 - (double)d->dropout;
    a.inv_keep = (float)(1.0 / keep);
    const double t = keep * 4294967296.0;
    a.thresh = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
    a.seed = d->seed;
    a.bf16 = d->dtype == 1;
    a.nqt = (a.Tq + MT - 1) / MT;
    a.nkt = (a.Tk + MT - 1) / MT;
    return 0;
}

static int hd_pad(int hd) { return hd <= 4 ? 4 : (hd <= 8 ? 8 : 16); }

// workspace: 256-byte aligned segments.  forward: K ext + V Z images; backward: delta, then
// K ext, K Z, V ext (key tiles) and Q ext, Q Z, dO ext, dO Z (query tiles)
struct MhaWs {
    size_t delta, kx, kz, vx, vz, qx, qz, gx, gz, total;
};
static MhaWs mha_ws_layout(const MhaArgs& a, bool bwd) {
    const int HDP = hd_pad(a.hd), TERMS = a.bf16 ? 1 : 3;
    const bool RS = TERMS == 3 && HDP <= 8;
    const int NX = (TERMS * HDP + 31) / 32, EW = (TERMS == 1 && HDP >= 8) ? HDP : 32 * NX,
              ZR = (TERMS == 1 && HDP >= 8) ? HDP : (TERMS == 1 ? 16 : (RS ? 16 : 32)), ZW = RS ? 128 : 64;
    const size_t bhn = (size_t)a.B * a.H, xt = (size_t)MT * EW * 2, zt = (size_t)ZR * ZW * 2;
    const size_t nk = bhn * ((a.Tk + MT - 1) / MT), nq = bhn * ((a.Tq + MT - 1) / MT);
    MhaWs w{};
    size_t off = 0;
    auto seg = [&](size_t bytes) {
        const size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    if (!bwd) {
        w.kx = seg(nk * xt);
        w.vz = seg(nk * zt);
    } else {
        w.delta = seg(bhn * a.Tq * sizeof(float));
        w.kx = seg(nk * xt);
        w.kz = seg(nk * zt);
        w.vx = seg(nk * xt);
        w.qx = seg(nq * xt);
        w.qz = seg(nq * zt);
        w.gx = seg(nq * xt);
        w.gz = seg(nq * zt);
    }
    w.total = off;
    return w;
}

template <int HDP, bool DROP, typename T>
static int mha_fwd_launch(MhaArgs& a, char* ws, hipStream_t s) {
    const MhaWs w = mha_ws_layout(a, false);
    uint16_t* kx = reinterpret_cast<uint16_t*>(ws + w.kx);
    uint16_t* vz = reinterpret_cast<uint16_t*>(ws + w.vz);
    SplitArgs sa{};
    sa.B = a.B; sa.H = a.H; sa.hd = a.hd;
    sa.op[0] = SplitOp{a.k, a.ks, a.Tk, a.nkt, 1.f, -1, kx, nullptr};
    sa.op[1] = SplitOp{a.v, a.vs, a.Tk, a.nkt, 1.f, (!DROP && a.hd < HDP) ? a.hd : -1, nullptr, vz};
    sa.nops = 2;
    mha_split_kernel<HDP, T><<<dim3(a.nkt, a.B * a.H), 256, 0, s>>>(sa);
    int rc = launch_status("mha_split");
    if (rc) return rc;
    a.kx = kx;
    a.vz = vz;
    dim3 grid(a.nqt, a.B * a.H);
    if (!DROP && a.hd < HDP) mha_fwd_mfma_kernel<HDP, DROP, T, true><<<grid, 256, 0, s>>>(a);
    else mha_fwd_mfma_kernel<HDP, DROP, T, false><<<grid, 256, 0, s>>>(a);
    return launch_status("mha_fwd");
}

template <int HDP, bool DROP, typename T>
static int mha_bwd_launch(MhaArgs& a, char* ws, hipStream_t s) {
    const MhaWs w = mha_ws_layout(a, true);
    a.delta = reinterpret_cast<float*>(ws + w.delta);
    auto img = [&](size_t off) { return reinterpret_cast<uint16_t*>(ws + off); };
    SplitArgs sa{};
    sa.B = a.B; sa.H = a.H; sa.hd = a.hd;
    sa.op[0] = SplitOp{a.k, a.ks, a.Tk, a.nkt, 1.f, -1, img(w.kx), img(w.kz)};
    sa.op[1] = SplitOp{a.v, a.vs, a.Tk, a.nkt, 1.f, -1, img(w.vx), nullptr};
    sa.op[2] = SplitOp{a.q, a.qs, a.Tq, a.nqt, a.scale2, -1, img(w.qx), img(w.qz)};
    sa.op[3] = SplitOp{a.dout, a.os, a.Tq, a.nqt, 1.f, -1, img(w.gx), img(w.gz)};
    sa.nops = 4;
    sa.o = a.o; sa.g = a.dout; sa.os = a.os; sa.Tq = a.Tq; sa.delta = a.delta;
    mha_split_kernel<HDP, T><<<dim3(a.nkt > a.nqt ? a.nkt : a.nqt, a.B * a.H), 256, 0, s>>>(sa);
    int rc = launch_status("mha_split");
    if (rc) return rc;
    a.kx = img(w.kx); a.kz = img(w.kz); a.vx = img(w.vx);
    a.qx = img(w.qx); a.qz = img(w.qz); a.gx = img(w.gx); a.gz = img(w.gz);
    constexpr int TERMS = kTerms<T>;
    const int lds = DqLds<HDP, TERMS>::BYTES > DkvLds<HDP, TERMS>::BYTES ? DqLds<HDP, TERMS>::BYTES
                                                                         : DkvLds<HDP, TERMS>::BYTES;
    mha_bwd_mfma_kernel<HDP, DROP, T><<<dim3(a.nkt > a.nqt ? a.nkt : a.nqt, a.B * a.H, 2),
                                         BwdRG<HDP, kTerms<T>>::NT, lds, s>>>(a);
    return launch_status("mha_bwd");
}

#define MMNI_MHA_DISPATCH_T(FN, T)                                                        \
    switch (hd_pad(a.hd)) {                                                               \
        case 4: return drop ? FN<4, true, T>(a, ws_, st_) : FN<4, false, T>(a, ws_, st_);   \
        case 8: return drop ? FN<8, true, T>(a, ws_, st_) : FN<8, false, T>(a, ws_, st_);   \
        default: return drop ? FN<16, true, T>(a, ws_, st_) : FN<16, false, T>(a, ws_, st_); \
    }
#define MMNI_MHA_DISPATCH(FN)                                                             \
    {                                                                                     \
        const bool drop = a.thresh != 0xffffffffu;                                        \
        hipStream_t st_ = (hipStream_t)stream;                                            \
        char* ws_ = static_cast<char*>(workspace);                                        \
        if (a.bf16) {                                                                     \
            MMNI_MHA_DISPATCH_T(FN, __bf16)                                               \
        } else {                                                                          \
            MMNI_MHA_DISPATCH_T(FN, float)                                                \
        }                                                                                 \
    }

}  // namespace mmni

using namespace mmni;

extern "C" size_t mmni_mha_fwd_workspace_bytes(const mmni_mha_desc* d) {
    MhaArgs a{};
    if (mha_fill(d, a)) return 0;
    return mha_ws_layout(a, false).total;
}

extern "C" size_t mmni_mha_bwd_workspace_bytes(const mmni_mha_desc* d) {
    MhaArgs a{};
    if (mha_fill(d, a)) return 0;
    return mha_ws_layout(a, true).total;
}

extern "C" int mmni_mha_fwd(const mmni_mha_desc* d, const void* q, const void* k, const void* v,
                            void* out, float* lse, void* workspace, void* stream) {
    MhaArgs a{};
    int rc = mha_fill(d, a);
    if (rc) return rc;
    MMNI_ARG_CHECK(q && k && v && out && lse && workspace, "mha_fwd: null pointer");
    MMNI_ARG_CHECK(reinterpret_cast<uintptr_t>(workspace) % 256 == 0, "mha_fwd: workspace must be 256-byte aligned");
    a.q = q; a.k = k; a.v = v; a.out = out; a.lse = lse;
    MMNI_MHA_DISPATCH(mha_fwd_launch)
}

extern "C" int mmni_mha_bwd(const mmni_mha_desc* d, const void* q, const void* k, const void* v,
                            const void* out, const void* dout, const float* lse, void* dq, void* dk,
                            void* dv, void* workspace, void* stream) {
    MhaArgs a{};
    int rc = mha_fill(d, a);
    if (rc) return rc;
    MMNI_ARG_CHECK(q && k && v && out && dout && lse && dq && dk && dv && workspace, "mha_bwd: null pointer");
    MMNI_ARG_CHECK(reinterpret_cast<uintptr_t>(workspace) % 256 == 0, "mha_bwd: workspace must be 256-byte aligned");
    a.q = q; a.k = k; a.v = v; a.o = out; a.dout = dout; a.lse = const_cast<float*>(lse);
    a.dq = dq; a.dk = dk; a.dv = dv;
    MMNI_MHA_DISPATCH(mha_bwd_launch)
}

extern "C" int mmni_mha_mean_probs(const mmni_mha_desc* d, const void* q, const void* k, const float* lse,
                                   float* probs, void* stream) {
    MhaArgs a{};
    int rc = mha_fill(d, a);
    if (rc) return rc;
    MMNI_ARG_CHECK(q && k && lse && probs, "mha_mean_probs: null pointer");
    a.q = q; a.k = k; a.lse = const_cast<float*>(lse); a.probs = probs;
    const int64_t n = (int64_t)a.B * a.Tq * a.Tk;
    if (a.thresh != 0xffffffffu)
        a.bf16 ? mha_probs_kernel<true, __bf16><<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(a)
               : mha_probs_kernel<true, float><<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(a);
    else
        a.bf16 ? mha_probs_kernel<false, __bf16><<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(a)
               : mha_probs_kernel<false, float><<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(a);
    return launch_status("mha_probs");
}

extern "C" int mmni_mha_dropout_mask(const mmni_mha_desc* d, float* mask, void* stream) {
    MhaArgs a{};
    int rc = mha_fill(d, a);
    if (rc) return rc;
    MMNI_ARG_CHECK(mask != nullptr, "mha_dropout_mask: null pointer");
    const int64_t n = (int64_t)a.B * a.H * a.Tq * a.Tk;
    mha_dropout_mask_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(a, mask);
    return launch_status("mha_dropout_mask");
}
