// Channels-last 3D convolutions for gfx950.
//
//   a4  PatchEmbed conv, kernel == stride, pad 0   modules/swin_v2_module.py:483,496
//       (3D lift: Conv3d(in, embed, k=s=patch))
//   a4b Conv k3 s1 p1 + LeakyReLU(0.2)             model.py:1195-1198,1331,1366-1368 in the
//       3D semantics of GreenBlock's Conv3d        nvidia_blocks.py:43,47
//
// Activations stay channels-last (B, D, H, W, C) — the token layout every Swin block uses —
// so the reference's patch_unembed / patch_embed transposes (swinfusion_module.py:971,1010)
// disappear.  Weights keep PyTorch's (Cout, Cin, k, k, k) layout.
//
// fwd : one lane per output voxel, all Cout accumulators in registers; weights are read with
//       wave-uniform addresses (scalar loads), input rows through L1/L2.  Bias and the
//       LeakyReLU are fused into the epilogue.
// dx  : one lane per input voxel (gather form of the transposed conv, no atomics).
// dw  : output tiles staged in LDS with their input halo; each lane owns (tap, cin) pairs
//       and all Cout accumulators; workgroups are persistent over tiles (a fixed tile set
//       per block) and write their partial dW/db to a workspace row; a fixed-order column
//       sum (tokenops.hip) reduces the rows, so dW/db are bitwise deterministic.
#include "mmni_common.h"

namespace mmni {

struct ConvArgs {
    int B, D, H, W, Cin, Cout, kd, kh, kw, sd, sh, sw, pd, ph, pw, Do, Ho, Wo;
    float slope;
    const float* x;
    const float* w;
    const float* bias;
    float* y;
    const float* dy;
    float* dx;
    float* dw;
    float* db;
    float* part;      // dw partials: [gridDim.x][Cout*Cin*K3 + Cout]
    // dw tiling
    int TZ, TY, TX, HZ, HY, HX, ntz, nty, ntx, ntiles;
};

__device__ __forceinline__ float lrelu_grad(float yv, float slope) { return yv > 0.f ? 1.f : slope; }

template <int CIN, int COUT>
__global__ __launch_bounds__(256) void conv3d_fwd_kernel(ConvArgs a) {
    const int64_t nvox = (int64_t)a.B * a.Do * a.Ho * a.Wo;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nvox) return;
    int64_t r = e;
    const int xo = (int)(r % a.Wo); r /= a.Wo;
    const int yo = (int)(r % a.Ho); r /= a.Ho;
    const int zo = (int)(r % a.Do);
    const int b = (int)(r / a.Do);
    float acc[COUT];
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[co] = a.bias ? a.bias[co] : 0.f;
    const int K3 = a.kd * a.kh * a.kw;
    const int z0 = zo * a.sd - a.pd, y0 = yo * a.sh - a.ph, x0 = xo * a.sw - a.pw;
    for (int tz = 0; tz < a.kd; ++tz) {
        const int z = z0 + tz;
        if (z < 0 || z >= a.D) continue;
        for (int ty = 0; ty < a.kh; ++ty) {
            const int y = y0 + ty;
            if (y < 0 || y >= a.H) continue;
            const float* xrow = a.x + (((int64_t)b * a.D + z) * a.H + y) * a.W * CIN;
            for (int tx = 0; tx < a.kw; ++tx) {
                const int xx = x0 + tx;
                if (xx < 0 || xx >= a.W) continue;
                const int t = (tz * a.kh + ty) * a.kw + tx;
                float xv[CIN];
#pragma unroll
                for (int ci = 0; ci < CIN; ++ci) xv[ci] = xrow[(int64_t)xx * CIN + ci];
#pragma unroll
                for (int co = 0; co < COUT; ++co) {
                    const float* wr = a.w + ((int64_t)co * CIN) * K3 + t;
                    float sacc = acc[co];
#pragma unroll
                    for (int ci = 0; ci < CIN; ++ci) sacc = fmaf(xv[ci], wr[(int64_t)ci * K3], sacc);
                    acc[co] = sacc;
                }
            }
        }
    }
    float* yo_p = a.y + e * COUT;
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
        const float v = acc[co];
        yo_p[co] = v > 0.f ? v : v * a.slope;
    }
}

// dx[v][ci] = sum_t sum_co dz[u(v,t)][co] * w[co][ci][t]
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void conv3d_dx_kernel(ConvArgs a) {
    const int64_t nvox = (int64_t)a.B * a.D * a.H * a.W;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nvox) return;
    int64_t r = e;
    const int x = (int)(r % a.W); r /= a.W;
    const int y = (int)(r % a.H); r /= a.H;
    const int z = (int)(r % a.D);
    const int b = (int)(r / a.D);
    float acc[CIN];
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) acc[ci] = 0.f;
    const int K3 = a.kd * a.kh * a.kw;
    for (int tz = 0; tz < a.kd; ++tz) {
        const int nz = z + a.pd - tz;
        if (nz < 0 || nz % a.sd) continue;
        const int uz = nz / a.sd;
        if (uz >= a.Do) continue;
        for (int ty = 0; ty < a.kh; ++ty) {
            const int ny = y + a.ph - ty;
            if (ny < 0 || ny % a.sh) continue;
            const int uy = ny / a.sh;
            if (uy >= a.Ho) continue;
            for (int tx = 0; tx < a.kw; ++tx) {
                const int nx = x + a.pw - tx;
                if (nx < 0 || nx % a.sw) continue;
                const int ux = nx / a.sw;
                if (ux >= a.Wo) continue;
                const int64_t u = (((int64_t)b * a.Do + uz) * a.Ho + uy) * a.Wo + ux;
                const int t = (tz * a.kh + ty) * a.kw + tx;
                float g[COUT];
#pragma unroll
                for (int co = 0; co < COUT; ++co) {
                    g[co] = a.dy[u * COUT + co];
                    if (a.slope != 1.f) g[co] *= lrelu_grad(a.y[u * COUT + co], a.slope);
                }
#pragma unroll
                for (int ci = 0; ci < CIN; ++ci) {
                    float sacc = acc[ci];
#pragma unroll
                    for (int co = 0; co < COUT; ++co)
                        sacc = fmaf(g[co], a.w[((int64_t)co * CIN + ci) * K3 + t], sacc);
                    acc[ci] = sacc;
                }
            }
        }
    }
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) a.dx[e * CIN + ci] = acc[ci];
}

// ------------------------------------------------------------------------------------
// k = 3, stride 1, pad 1 (the a4b convs): LDS-tiled stencil for the forward and dx
// ------------------------------------------------------------------------------------
// One workgroup = an 8 x 8 x 4 tile of output voxels (one per lane).  The tile's input halo
// (10 x 10 x 6 rows of NI channels) is staged in LDS once, so each input row is read from HBM
// ~1.7x instead of once per tap through L2 (the gather kernels above re-read 19-21 GB per dx
// launch at 96^3).  Weights are wave-uniform (scalar loads).
//   MODE 0 (forward):  out[v][o] = bias[o] + sum_t sum_i x[v + t - 1][i] * w[o][i][t], LeakyReLU
//   MODE 1 (dx):       dx[v][i]  = sum_t sum_o dz[v + 1 - t][o] * w[o][i][t],
//                      dz = dy * LeakyReLU'(y) computed once per halo row while staging.
constexpr int kDwBlocksPerCU = 8;   // dW kernel: persistent blocks per CU (each flushes its partials once)
constexpr int kTX = 8, kTY = 8, kTZ = 4;
constexpr int kHX = kTX + 2, kHY = kTY + 2, kHZ = kTZ + 2;

// LDS row stride of NI floats: whole float4 chunks, an odd number of them (bank spread)
template <int NI>
struct HaloRow {
    static constexpr int kChunks0 = (NI + 3) / 4;
    static constexpr int kChunks = NI < 4 ? 0 : (kChunks0 % 2 ? kChunks0 : kChunks0 + 1);
    static constexpr int kStride = NI < 4 ? NI : kChunks * 4;
};

template <int CIN, int COUT, int MODE>
__global__ __launch_bounds__(256) void conv3d_k3_tile_kernel(ConvArgs a) {
    constexpr int NI = MODE == 0 ? CIN : COUT;   // channels of the staged operand
    constexpr int NO = MODE == 0 ? COUT : CIN;   // channels of the result
    constexpr int RS = HaloRow<NI>::kStride;
    __shared__ __attribute__((aligned(16))) float halo[kHX * kHY * kHZ * RS];
    const int ntx = (a.W + kTX - 1) / kTX, nty = (a.H + kTY - 1) / kTY, ntz = (a.D + kTZ - 1) / kTZ;
    int tile = blockIdx.x;
    const int bx = tile % ntx; tile /= ntx;
    const int by = tile % nty; tile /= nty;
    const int bz = tile % ntz;
    const int b = tile / ntz;
    const int x0 = bx * kTX - 1, y0 = by * kTY - 1, z0 = bz * kTZ - 1;
    const float* src = MODE == 0 ? a.x : a.dy;
    // ---- stage the halo (zero outside the volume)
    for (int e = threadIdx.x; e < kHX * kHY * kHZ; e += 256) {
        const int hx = e % kHX, hy = (e / kHX) % kHY, hz = e / (kHX * kHY);
        const int gx = x0 + hx, gy = y0 + hy, gz = z0 + hz;
        float v[NI];
        const bool in = gx >= 0 && gx < a.W && gy >= 0 && gy < a.H && gz >= 0 && gz < a.D;
        const int64_t row = in ? (((int64_t)b * a.D + gz) * a.H + gy) * a.W + gx : 0;
        if (NI % 4 == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
            // 16-B rows: float4 loads (NI / 4 per row instead of NI)
#pragma unroll
            for (int c = 0; c < (NI % 4 == 0 ? NI : 0); c += 4) {
                const float4 q = in ? *reinterpret_cast<const float4*>(src + row * NI + c) : make_float4(0.f, 0.f, 0.f, 0.f);
                v[c] = q.x; v[c + 1] = q.y; v[c + 2] = q.z; v[c + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int c = 0; c < NI; ++c) v[c] = in ? src[row * NI + c] : 0.f;
        }
        if (MODE == 1 && in && a.slope != 1.f) {
#pragma unroll
            for (int c = 0; c < NI; ++c) v[c] *= lrelu_grad(a.y[row * NI + c], a.slope);
        }
        float* dst = halo + e * RS;
        if constexpr (RS % 4 == 0) {
#pragma unroll
            for (int c = 0; c < RS; c += 4)
                *reinterpret_cast<float4*>(dst + c) = make_float4(c < NI ? v[c] : 0.f, c + 1 < NI ? v[c + 1] : 0.f,
                                                                  c + 2 < NI ? v[c + 2] : 0.f, c + 3 < NI ? v[c + 3] : 0.f);
        } else {
#pragma unroll
            for (int c = 0; c < NI; ++c) dst[c] = v[c];
        }
    }
    __syncthreads();
    const int tx = threadIdx.x & 7, ty = (threadIdx.x >> 3) & 7, tz = threadIdx.x >> 6;
    float acc[NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) acc[o] = (MODE == 0 && a.bias) ? a.bias[o] : 0.f;
    // Tap-inner order: for one staged channel i, the 27 tap values come from LDS, and the weights of
    // one (i, o) pair are 27 consecutive floats (PyTorch layout, t fastest), fetched with a few wide
    // scalar loads.  The tap-outer order below issues one s_load_dword plus a 64-bit address add per
    // weight (~6 SALU per VALU FMA pair at 24 -> 12: scalar-issue bound).
    const float* hb = halo + ((tz * kHY + ty) * kHX + tx) * RS;
    // Channels in pairs (i0 even, NI even, 8-B aligned weights): a run (ci, co) of 27 weights then
    // starts at an even or odd float by a compile-time rule, so its taps go to v_pk_fma_f32 as
    // 8-B aligned pairs (aligned SGPR pairs, no realigning moves); the odd tap is a scalar FMA.
    // (forward only: the dx tile, 24 outputs per lane, measured slower paired: 2.77 vs 2.59 ms at 24 -> 12)
    constexpr int IS = (MODE == 0 && NI % 2 == 0) ? 2 : 1;
    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll 1
    for (int i0 = 0; i0 < NI; i0 += IS) {
#pragma unroll
        for (int si = 0; si < IS; ++si) {
            const int i = i0 + si;
            float xv[27];
#pragma unroll
            for (int t = 0; t < 27; ++t) {
                const int kz = t / 9, ky = (t / 3) % 3, kx = t % 3;
                const int hz = MODE == 0 ? kz : 2 - kz, hy = MODE == 0 ? ky : 2 - ky, hx = MODE == 0 ? kx : 2 - kx;
                xv[t] = hb[((hz * kHY + hy) * kHX + hx) * RS + i];
            }
#pragma unroll
            for (int o = 0; o < NO; ++o) {
                const float* wp = a.w + (MODE == 0 ? (o * CIN + i) : (i * CIN + o)) * 27;
                if (IS == 2) {
                    // one run's weights in SGPRs at a time (hoisting them all spills SGPRs to VGPR lanes)
                    __builtin_amdgcn_sched_barrier(0);
                    // parity of the run start (i0 even): MODE 0 (o*CIN + si)*27, MODE 1 (si*CIN + o)*27
                    const int par = (MODE == 0 ? (o * CIN + si) : (si * CIN + o)) & 1;
                    f2 a2 = (f2){0.f, 0.f};
                    float sacc = acc[o];
                    if (par == 0) {
#pragma unroll
                        for (int t = 0; t < 26; t += 2)
                            a2 = __builtin_elementwise_fma((f2){xv[t], xv[t + 1]},
                                                           *reinterpret_cast<const f2*>(wp + t), a2);
                        sacc = fmaf(xv[26], wp[26], sacc);
                    } else {
                        sacc = fmaf(xv[0], wp[0], sacc);
#pragma unroll
                        for (int t = 1; t < 27; t += 2)
                            a2 = __builtin_elementwise_fma((f2){xv[t], xv[t + 1]},
                                                           *reinterpret_cast<const f2*>(wp + t), a2);
                    }
                    acc[o] = sacc + (a2.x + a2.y);
                } else {
                    float sacc = acc[o];
#pragma unroll
                    for (int t = 0; t < 27; ++t) sacc = fmaf(xv[t], wp[t], sacc);
                    acc[o] = sacc;
                }
            }
        }
    }
    const int gx = bx * kTX + tx, gy = by * kTY + ty, gz = bz * kTZ + tz;
    if (gx >= a.W || gy >= a.H || gz >= a.D) return;
    const int64_t vox = (((int64_t)b * a.D + gz) * a.H + gy) * a.W + gx;
    float* out = (MODE == 0 ? a.y : a.dx) + vox * NO;
#pragma unroll
    for (int o = 0; o < NO; ++o) out[o] = MODE == 0 ? (acc[o] > 0.f ? acc[o] : acc[o] * a.slope) : acc[o];
}

__host__ __forceinline__ bool is_k3_same(const ConvArgs& a) {
    return a.kd == 3 && a.kh == 3 && a.kw == 3 && a.sd == 1 && a.sh == 1 && a.sw == 1 && a.pd == 1 && a.ph == 1 &&
           a.pw == 1 && a.Do == a.D && a.Ho == a.H && a.Wo == a.W;
}

__host__ __forceinline__ unsigned k3_tiles(const ConvArgs& a) {
    return (unsigned)((int64_t)a.B * ((a.D + kTZ - 1) / kTZ) * ((a.H + kTY - 1) / kTY) * ((a.W + kTX - 1) / kTX));
}

// dW[co][ci][t] += sum_u dz[u][co] * x[in(u,t)][ci];  db[co] += sum_u dz[u][co]
template <int CIN, int COUT, int MAXP>
__global__ __launch_bounds__(256) void conv3d_dw_kernel(ConvArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int K3 = a.kd * a.kh * a.kw;
    const int npairs = K3 * CIN;
    const int Tout = a.TZ * a.TY * a.TX;
    const int Tin = a.HZ * a.HY * a.HX;
    float* dz_s = smem;                       // [Tout][COUT]
    float* x_s = dz_s + Tout * COUT;          // [Tin][CIN]
    const int tid = threadIdx.x;
    float acc[MAXP][COUT];
    float dbl[COUT];   // db partial: sum of the dz rows this thread staged (any COUT vs npairs)
#pragma unroll
    for (int co = 0; co < COUT; ++co) dbl[co] = 0.f;
#pragma unroll
    for (int m = 0; m < MAXP; ++m)
#pragma unroll
        for (int co = 0; co < COUT; ++co) acc[m][co] = 0.f;
    const int tiles_per_b = a.ntz * a.nty * a.ntx;
    const int G = MAXP == 1 ? (256 / npairs > 0 ? 256 / npairs : 1) : 1;   // lane groups over voxels
    const int gi = MAXP == 1 ? tid / npairs : 0;
    const int pl = MAXP == 1 ? tid - gi * npairs : tid;
    // x_s offset of each owned pair relative to the voxel's halo base
    int xo[MAXP];
#pragma unroll
    for (int m = 0; m < MAXP; ++m) {
        const int p = pl + m * 256;
        const int pv = p < npairs ? p : 0;
        const int ci = pv % CIN, t = pv / CIN;
        const int tx = t % a.kw, ty = (t / a.kw) % a.kh, tz = t / (a.kw * a.kh);
        xo[m] = ((tz * a.HY + ty) * a.HX + tx) * CIN + ci;
    }

    for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
        int rr = tile;
        const int bx = rr % a.ntx; rr /= a.ntx;
        const int by = rr % a.nty; rr /= a.nty;
        const int bz = rr % a.ntz;
        const int b = rr / a.ntz;
        (void)tiles_per_b;
        const int oz0 = bz * a.TZ, oy0 = by * a.TY, ox0 = bx * a.TX;
        const int iz0 = oz0 * a.sd - a.pd, iy0 = oy0 * a.sh - a.ph, ix0 = ox0 * a.sw - a.pw;
        __syncthreads();
        for (int e = tid; e < Tout; e += blockDim.x) {
            const int lx = e % a.TX, ly = (e / a.TX) % a.TY, lz = e / (a.TX * a.TY);
            const int oz = oz0 + lz, oy = oy0 + ly, ox = ox0 + lx;
            float g[COUT];
            if (oz < a.Do && oy < a.Ho && ox < a.Wo) {
                const int64_t u = (((int64_t)b * a.Do + oz) * a.Ho + oy) * a.Wo + ox;
#pragma unroll
                for (int co = 0; co < COUT; ++co) {
                    g[co] = a.dy[u * COUT + co];
                    if (a.slope != 1.f) g[co] *= lrelu_grad(a.y[u * COUT + co], a.slope);
                }
            } else {
#pragma unroll
                for (int co = 0; co < COUT; ++co) g[co] = 0.f;
            }
#pragma unroll
            for (int co = 0; co < COUT; ++co) {
                dz_s[e * COUT + co] = g[co];
                dbl[co] += g[co];
            }
        }
        // halo rows as float4 chunks when rows are 16-B multiples: the index math runs per chunk
        const bool vec4 = CIN % 4 == 0 && (Tout * COUT) % 4 == 0 && reinterpret_cast<uintptr_t>(a.x) % 16 == 0;
        if (vec4) {
            constexpr int C4 = CIN / 4 > 0 ? CIN / 4 : 1;
            for (int e = tid; e < Tin * C4; e += blockDim.x) {
                const int c4 = e % C4, v = e / C4;
                const int lx = v % a.HX, ly = (v / a.HX) % a.HY, lz = v / (a.HX * a.HY);
                const int z = iz0 + lz, y = iy0 + ly, x = ix0 + lx;
                float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (z >= 0 && z < a.D && y >= 0 && y < a.H && x >= 0 && x < a.W)
                    xv = *reinterpret_cast<const float4*>(a.x + ((((int64_t)b * a.D + z) * a.H + y) * a.W + x) * CIN +
                                                          4 * c4);
                *reinterpret_cast<float4*>(x_s + v * CIN + 4 * c4) = xv;
            }
        }
        for (int e = tid; e < (vec4 ? 0 : Tin * CIN); e += blockDim.x) {
            const int ci = e % CIN, v = e / CIN;
            const int lx = v % a.HX, ly = (v / a.HX) % a.HY, lz = v / (a.HX * a.HY);
            const int z = iz0 + lz, y = iy0 + ly, x = ix0 + lx;
            float xv = 0.f;
            if (z >= 0 && z < a.D && y >= 0 && y < a.H && x >= 0 && x < a.W)
                xv = a.x[((((int64_t)b * a.D + z) * a.H + y) * a.W + x) * CIN + ci];
            x_s[e] = xv;
        }
        __syncthreads();
        // pair (t, ci) owned by this lane: p = tid + m*256; with fewer pairs than lanes (MAXP 1)
        // the block splits into G groups of npairs lanes that take every G-th output voxel.
        // Lanes past the last pair (or group) compute on pair 0 and are dropped at the flush, so
        // the loop has no per-pair branch; the voxel coordinates advance without divisions.
        int ux = gi % a.TX, uy = (gi / a.TX) % a.TY, uz = gi / (a.TX * a.TY);
        for (int u = gi; u < Tout; u += G) {
            const int hb = ((uz * a.sd * a.HY) + uy * a.sh) * a.HX + ux * a.sw;
            float g[COUT];
#pragma unroll
            for (int co = 0; co < COUT; ++co) g[co] = dz_s[u * COUT + co];
#pragma unroll
            for (int m = 0; m < MAXP; ++m) {
                const float xv = x_s[hb * CIN + xo[m]];
#pragma unroll
                for (int co = 0; co < COUT; ++co) acc[m][co] = fmaf(g[co], xv, acc[m][co]);
            }
            ux += G;
            while (ux >= a.TX) {
                ux -= a.TX;
                if (++uy == a.TY) { uy = 0; ++uz; }
            }
        }
    }
    // lane groups (MAXP 1, G > 1): sum the G partials of a pair through LDS in group order, so
    // the block's partial row is written once per (pair, co)
    bool flush = gi < G;
    if (MAXP == 1 && G > 1) {
        __syncthreads();
        float* red = smem;                        // [G][npairs][COUT]
        if (gi < G) {
#pragma unroll
            for (int co = 0; co < COUT; ++co) red[(gi * npairs + pl) * COUT + co] = acc[0][co];
        }
        __syncthreads();
        if (gi == 0) {
#pragma unroll
            for (int co = 0; co < COUT; ++co) {
                float sum = 0.f;
                for (int q = 0; q < G; ++q) sum += red[(q * npairs + pl) * COUT + co];
                acc[0][co] = sum;
            }
        }
        flush = gi == 0;
    }
    // this block's partial row; every column is written by exactly one lane of every block
    const int ncw = npairs * COUT;
    float* row = a.part + (int64_t)blockIdx.x * (ncw + COUT);
#pragma unroll
    for (int m = 0; m < MAXP; ++m) {
        const int p = pl + m * 256;
        if (p < npairs && flush) {
            const int ci = p % CIN, t = p / CIN;
#pragma unroll
            for (int co = 0; co < COUT; ++co) row[((int64_t)co * CIN + ci) * K3 + t] = acc[m][co];
        }
    }
    // db: the 256 per-thread sums, reduced in a fixed order by lanes co < COUT
    __syncthreads();
    float* redd = smem;   // [COUT][256]
#pragma unroll
    for (int co = 0; co < COUT; ++co) redd[co * 256 + tid] = dbl[co];
    __syncthreads();
    if (tid < COUT) {
        float sum = 0.f;
        for (int q = 0; q < 256; ++q) sum += redd[tid * 256 + q];
        row[ncw + tid] = sum;
    }
}

static int conv_fill(const mmni_conv3d_desc* d, ConvArgs& a) {
    MMNI_ARG_CHECK(d != nullptr, "conv3d: null descriptor");
    MMNI_ARG_CHECK(d->B > 0 && d->D > 0 && d->H > 0 && d->W > 0 && d->Cin > 0 && d->Cout > 0, "conv3d: bad sizes");
    MMNI_ARG_CHECK(d->kd > 0 && d->kh > 0 && d->kw > 0 && d->sd > 0 && d->sh > 0 && d->sw > 0 && d->pd >= 0 &&
                       d->ph >= 0 && d->pw >= 0,
                   "conv3d: bad kernel/stride/pad");
    auto osz = [](int n, int k, int s, int p) { return (n + 2 * p - k) / s + 1; };
    MMNI_ARG_CHECK(d->Do == osz(d->D, d->kd, d->sd, d->pd) && d->Ho == osz(d->H, d->kh, d->sh, d->ph) &&
                       d->Wo == osz(d->W, d->kw, d->sw, d->pw) && d->Do > 0 && d->Ho > 0 && d->Wo > 0,
                   "conv3d: output extents (%d,%d,%d) inconsistent with input/kernel", d->Do, d->Ho, d->Wo);
    a.B = d->B; a.D = d->D; a.H = d->H; a.W = d->W; a.Cin = d->Cin; a.Cout = d->Cout;
    a.kd = d->kd; a.kh = d->kh; a.kw = d->kw; a.sd = d->sd; a.sh = d->sh; a.sw = d->sw;
    a.pd = d->pd; a.ph = d->ph; a.pw = d->pw;
    a.Do = d->Do; a.Ho = d->Ho; a.Wo = d->Wo;
    a.slope = d->slope;
    return 0;
}

// dW tiling plan: output tile (TZ, TY, TX) shrunk until the LDS image (dz tile + input halo)
// fits 64 KiB; persistent grid of at most kNumCU * kDwBlocksPerCU blocks.
static int dw_plan(ConvArgs& a, int& grid, size_t& lds) {
    const int CIN = a.Cin, COUT = a.Cout;
    int TZ = 4, TY = 4, TX = 16;
    auto hz = [&](int T) { return (T - 1) * a.sd + a.kd; };
    auto hy = [&](int T) { return (T - 1) * a.sh + a.kh; };
    auto hx = [&](int T) { return (T - 1) * a.sw + a.kw; };
    if (a.Do == 1) TZ = 1;
    auto bytes = [&]() {
        return (size_t)(TZ * TY * TX * COUT + hz(TZ) * hy(TY) * hx(TX) * CIN) * 4;
    };
    while (bytes() > 64 * 1024) {
        if (TX > 4) TX /= 2;
        else if (TY > 1) TY /= 2;
        else if (TZ > 1) TZ /= 2;
        else if (TX > 1) TX /= 2;
        else break;
    }
    MMNI_ARG_CHECK(bytes() <= 64 * 1024, "conv3d_dw: kernel too large for the LDS tile");
    a.TZ = TZ; a.TY = TY; a.TX = TX;
    a.HZ = hz(TZ); a.HY = hy(TY); a.HX = hx(TX);
    a.ntz = (a.Do + TZ - 1) / TZ; a.nty = (a.Ho + TY - 1) / TY; a.ntx = (a.Wo + TX - 1) / TX;
    a.ntiles = a.B * a.ntz * a.nty * a.ntx;
    const int npairs = a.kd * a.kh * a.kw * CIN;
    MMNI_ARG_CHECK(npairs <= 1024, "conv3d_dw: k^3*Cin = %d exceeds 1024 pairs", npairs);
    grid = a.ntiles < kNumCU * kDwBlocksPerCU ? a.ntiles : kNumCU * kDwBlocksPerCU;
    // the group reduction of the MAXP 1 kernel ([G][npairs][COUT]) and the db reduction
    // ([COUT][256]) reuse the LDS image
    const int G = npairs <= 256 ? (256 / npairs > 0 ? 256 / npairs : 1) : 1;
    size_t red = (size_t)G * npairs * COUT * 4;
    if (red < (size_t)256 * COUT * 4) red = (size_t)256 * COUT * 4;
    lds = bytes() > red ? bytes() : red;
    MMNI_ARG_CHECK(lds <= 64 * 1024, "conv3d_dw: group reduction exceeds the LDS tile");
    return 0;
}

template <int CIN, int COUT>
static int conv_fwd_launch(ConvArgs& a, hipStream_t s) {
    // every k3 same-padding forward takes the LDS tile (tap-inner weights: faster than the lane-per-
    // voxel gather at every channel pair since r10); other geometries (k = s = p) the gather
    if (is_k3_same(a)) {
        MMNI_ARG_CHECK(reinterpret_cast<uintptr_t>(a.w) % 8 == 0, "conv3d_fwd: k3 weights must be 8-byte aligned");
        conv3d_k3_tile_kernel<CIN, COUT, 0><<<k3_tiles(a), 256, 0, s>>>(a);
        return launch_status("conv3d_fwd_k3");
    }
    const int64_t n = (int64_t)a.B * a.Do * a.Ho * a.Wo;
    conv3d_fwd_kernel<CIN, COUT><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a);
    return launch_status("conv3d_fwd");
}

template <int CIN, int COUT>
static int conv_bwd_launch(ConvArgs& a, hipStream_t s) {
    if (a.dx && is_k3_same(a)) {
        conv3d_k3_tile_kernel<CIN, COUT, 1><<<k3_tiles(a), 256, 0, s>>>(a);
        int rc = launch_status("conv3d_dx_k3");
        if (rc) return rc;
    } else if (a.dx) {
        const int64_t n = (int64_t)a.B * a.D * a.H * a.W;
        conv3d_dx_kernel<CIN, COUT><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a);
        int rc = launch_status("conv3d_dx");
        if (rc) return rc;
    }
    int grid;
    size_t lds;
    int rc = dw_plan(a, grid, lds);
    if (rc) return rc;
    MMNI_ARG_CHECK(a.part != nullptr, "conv3d_bwd: null workspace");
    const int npairs = a.kd * a.kh * a.kw * CIN;
#define MMNI_DW(MP)                                                                            \
    conv3d_dw_kernel<CIN, COUT, MP><<<grid, 256, lds, s>>>(a);                                 \
    rc = launch_status("conv3d_dw");                                                           \
    if (rc) return rc;                                                                         \
    column_sum(a.part, grid, npairs * COUT + COUT, a.dw, npairs * COUT, a.db, s);              \
    return launch_status("conv3d_dw_colsum");
    if (npairs <= 256) { MMNI_DW(1) }
    if (npairs <= 512) { MMNI_DW(2) }
    if (npairs <= 768) { MMNI_DW(3) }
    if (npairs <= 1024) { MMNI_DW(4) }
#undef MMNI_DW
    set_error("conv3d_dw: k^3*Cin = %d exceeds 1024 pairs", npairs);
    return -2;
}

#define MMNI_CONV_DISPATCH(FN)                                                               \
    {                                                                                        \
        const int ci = a.Cin, co = a.Cout;                                                  \
        hipStream_t st = (hipStream_t)stream;                                                \
        if (ci == 1 && co == 12) return FN<1, 12>(a, st);                                    \
        if (ci == 1 && co == 6) return FN<1, 6>(a, st);                                      \
        if (ci == 6 && co == 12) return FN<6, 12>(a, st);                                    \
        if (ci == 6 && co == 6) return FN<6, 6>(a, st);                                      \
        if (ci == 24 && co == 12) return FN<24, 12>(a, st);                                  \
        if (ci == 12 && co == 12) return FN<12, 12>(a, st);                                  \
        if (ci == 12 && co == 6) return FN<12, 6>(a, st);                                    \
        if (ci == 6 && co == 3) return FN<6, 3>(a, st);                                      \
        if (ci == 3 && co == 1) return FN<3, 1>(a, st);                                      \
        if (ci == 2 && co == 4) return FN<2, 4>(a, st);                                      \
        set_error("conv3d: unsupported (Cin=%d, Cout=%d)", ci, co);                          \
        return -2;                                                                           \
    }

}  // namespace mmni

using namespace mmni;

extern "C" int mmni_conv3d_fwd(const mmni_conv3d_desc* d, const float* x, const float* w, const float* bias,
                               float* y, void* stream) {
    ConvArgs a{};
    int rc = conv_fill(d, a);
    if (rc) return rc;
    MMNI_ARG_CHECK(x && w && y, "conv3d_fwd: null pointer");
    a.x = x; a.w = w; a.bias = bias; a.y = y;
    MMNI_CONV_DISPATCH(conv_fwd_launch)
}

extern "C" size_t mmni_conv3d_bwd_workspace_bytes(const mmni_conv3d_desc* d) {
    ConvArgs a{};
    if (conv_fill(d, a)) return 0;
    int grid;
    size_t lds;
    if (dw_plan(a, grid, lds)) return 0;
    return (size_t)grid * (a.kd * a.kh * a.kw * a.Cin * a.Cout + a.Cout) * sizeof(float);
}

extern "C" int mmni_conv3d_bwd(const mmni_conv3d_desc* d, const float* x, const float* w, const float* y,
                               const float* dy, float* dx, float* dw, float* db, void* workspace, void* stream) {
    ConvArgs a{};
    int rc = conv_fill(d, a);
    if (rc) return rc;
    a.part = static_cast<float*>(workspace);
    MMNI_ARG_CHECK(x && w && dy && dw, "conv3d_bwd: null pointer");
    MMNI_ARG_CHECK(d->slope == 1.f || y != nullptr, "conv3d_bwd: LeakyReLU gradient needs y");
    a.x = x; a.w = w; a.y = const_cast<float*>(y); a.dy = dy; a.dx = dx; a.dw = dw; a.db = db;
    MMNI_CONV_DISPATCH(conv_bwd_launch)
}
