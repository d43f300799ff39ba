// Complex-valued MLP training step on the matrix cores (gfx950 MFMA).
//
// The same step as cvnn.hip (reference cvnn.py:65-210 ComplexLinear / modReLU / zReLU,
// gbm_trainer.py:819-835 spectral MSE + backward), with every product a real GEMM on MFMA:
//
//   * a complex layer y = W z + b (W = A + iB, z = x + iy) is the real map of the interleaved
//     vectors Z = (x0, y0, x1, y1, ...):  Wc[2j + a][2k + b] = [[A, -B], [B, A]]_{jk}[a][b],
//     so U = Z Wc^T (features (u_j, v_j) interleaved, the complex64 layout of the targets),
//     dZ = dU Wc, dWc = dU^T Z; dA = dWc[2j][2k] + dWc[2j+1][2k+1], dB = dWc[2j+1][2k] - dWc[2j][2k+1];
//     the bias gradients are the extra "ones" column 2 ni of Z in the weight-gradient GEMM.
//   * operand types (SMC_CVNN_MFMA_F32 / SMC_CVNN_MFMA_BF16):
//       f32:  v_mfma_f32_16x16x4_f32   (exact f32 fma chains, the network's own dtype)
//       bf16: v_mfma_f32_16x16x32_bf16 (bf16 operands rounded to nearest even, f32 accumulate;
//             master parameters, activations, loss, Adam stay f32 — BASELINE configs[2] extension;
//             the reference itself asserts full precision, gbm_trainer.py:679-686)
//
// Launches per step (all stream-ordered, no atomics, fixed reduction orders: bit-reproducible):
//   pack_kernel       Wc [W_out][W_in] and Wc^T [W_in][W_out] of every layer from the f32 params
//   fb_kernel         16 * RT batch rows per workgroup: forward through every layer (GEMM + bias +
//                     activation epilogue, activations in LDS), loss and output gradient, then the
//                     input-gradient GEMMs down the layers with the activation backward fused in
//                     their epilogue.  Writes Z_l^T and dU_l^T ([feature][batch]) for the weight
//                     gradients, modReLU-bias and loss partials per workgroup.
//   wgrad_kernel      dWc_l = dU_l^T Z_l per (feature tile, column-tile group, batch segment), one wave
//                     per item, K = the segment's batch rows; writes partials[segment][n_params + 1]
//                     (weights, biases, modReLU biases, loss), which smc_cvnn_reduce_grads sums in order.
//
// MFMA fragments (MI355X / CDNA4): lane l = 16 g + c supplies 16 bytes of A row c and of B column c
// at K offset g * KB / 4 of the K block; C/D: lane l holds rows 4 g .. 4 g + 3 of column c.  In the
// f32 form the four instructions of a K block take element i of each lane's 4-vector, so a block
// covers k = kb + 4 g + i for g, i in 0..3 on A and B alike.
#include <cmath>

#include "smc_device.h"
#include "smc_internal.h"

namespace smc {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxL = SMC_CVNN_MAX_LAYERS;
constexpr int kMaxSegments = 64;     // batch segments of the weight-gradient GEMMs
constexpr int kSegmentRows = 256;    // minimum rows per segment
constexpr int64_t kWgradBlocks = 2048;  // segments are added until the workgroups reach this
constexpr size_t kLdsCap = 156 * 1024;   // dynamic LDS of fb_kernel (160 KiB per CU, less its static LDS)
constexpr size_t kLdsPair = 80 * 1024;   // two row tiles per workgroup only within this


struct OpBf16 {
  using T = uint16_t;
  using V = bf16x8;
  static constexpr int KB = 32;  // one v_mfma_f32_16x16x32_bf16 per K block
  static __device__ __forceinline__ T cvt(float x) { return bf16_bits(x); }
  static __device__ __forceinline__ V ld(const T* p) { return *reinterpret_cast<const V*>(p); }
  static __device__ __forceinline__ f32x4 mmav(f32x4 acc, V a, V b) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x4 mma(f32x4 acc, const T* a, const T* b) {
    const bf16x8 av = *reinterpret_cast<const bf16x8*>(a);
    const bf16x8 bv = *reinterpret_cast<const bf16x8*>(b);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  }
  static __device__ __forceinline__ void store4(T* p, float a, float b, float c, float d) {
    *reinterpret_cast<u16x4*>(p) = u16x4{cvt(a), cvt(b), cvt(c), cvt(d)};
  }
};

struct OpF32 {
  using T = float;
  using V = f32x4;
  static constexpr int KB = 16;  // four v_mfma_f32_16x16x4_f32 per K block
  static __device__ __forceinline__ T cvt(float x) { return x; }
  static __device__ __forceinline__ V ld(const T* p) { return *reinterpret_cast<const V*>(p); }
  static __device__ __forceinline__ f32x4 mmav(f32x4 acc, V a, V b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], acc, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x4 mma(f32x4 acc, const T* a, const T* b) {
    const f32x4 av = *reinterpret_cast<const f32x4*>(a);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(b);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1], bv[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[2], bv[2], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x4f32(av[3], bv[3], acc, 0, 0, 0);
  }
  static __device__ __forceinline__ void store4(T* p, float a, float b, float c, float d) {
    *reinterpret_cast<f32x4*>(p) = f32x4{a, b, c, d};
  }
};

// Per-layer plan (host-computed).  W_in = roundup(2 ni, KB), W_out = roundup(2 no, KB).
struct MLayer {
  int32_t ni, no, act, win, wout, kx;  // kx = roundup(2 ni + 1, 16): rows of Z^T (ones row at 2 ni)
  int64_t w_re, w_im, b_re, b_im, act_bias;
  int64_t wc, wct;   // Op offsets: Wc [wout][win] (layered: [wout][kx] with the bias column at 2 ni), Wc^T [win][wout]
  int64_t zt, gt;    // Op offsets: Z^T [kx][bp], dU^T [wout][bp]
  int64_t zr, dr;    // layered only: Z [bp][kx], dU [bp][wout] (row-major GEMM operands)
  int64_t pre;       // f32 offset of the pre-activation [R][2 no] in the workgroup's LDS (hidden layers
                     // with an activation), or -1
  int64_t cpart;     // f32 offset of the modReLU-bias partials [nwg][no], or -1
  int64_t items;     // weight-gradient items (waves) of this layer, all segments
};

struct MArgs {
  int32_t n_layers;
  MLayer layer[kMaxL];
  int64_t batch, bp;
  int32_t rows;      // batch rows per fb workgroup (16 RT)
  int32_t nwg;       // fb workgroups = bp / rows
  int32_t segs;      // batch segments of the weight gradients
  int32_t zs, gs;    // LDS row strides (Op elements) of the activation and output-gradient buffers
  int32_t pre_global;  // pre-activations in the f32 workspace [bp][2 no] instead of LDS [R][2 no]
  int32_t lgemm_mb;  // lgemm_kernel launches: feature blocks of the launch (set per launch)
  int32_t layered;   // wide layers: one MFMA GEMM launch per layer and direction (lgemm_kernel) instead of fb_kernel
  int32_t lpb;       // loss partials per batch block of `rows` rows (1; layered: feature blocks of the last layer)
  int64_t n_params;
  int64_t pack_elems;
  const float* params;
  const float* in_re;
  const float* in_im;
  const float* targets;   // [batch][N] complex64
  void* opws;
  float* fws;
  double* lossp;          // [nwg]
  float* partials;        // [segs][n_params + 1]
};

// ---- pack ------------------------------------------------------------------------------------
template <class Op>
__global__ __launch_bounds__(kThreads) void pack_kernel(MArgs a) {
  using T = typename Op::T;
  T* ws = static_cast<T*>(a.opws);
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; e < a.pack_elems;
       e += static_cast<int64_t>(gridDim.x) * kThreads) {
    int64_t r = e;
    int l = 0;
    while (r >= 2LL * a.layer[l].wout * a.layer[l].win) {
      r -= 2LL * a.layer[l].wout * a.layer[l].win;
      ++l;
    }
    const MLayer& ly = a.layer[l];
    const int64_t n = static_cast<int64_t>(ly.wout) * ly.win;
    const bool transposed = r >= n;
    if (transposed) r -= n;
    const int f = transposed ? static_cast<int>(r % ly.wout) : static_cast<int>(r / ly.win);
    const int k = transposed ? static_cast<int>(r / ly.wout) : static_cast<int>(r % ly.win);
    const int j = f >> 1, kk = k >> 1, ra = f & 1, rb = k & 1;
    float v = 0.0f;
    if (j < ly.no && kk < ly.ni) {
      const float wa = a.params[ly.w_re + static_cast<int64_t>(j) * ly.ni + kk];
      const float wb = a.params[ly.w_im + static_cast<int64_t>(j) * ly.ni + kk];
      v = ra == rb ? wa : (ra == 0 ? -wb : wb);
    }
    ws[(transposed ? ly.wct : ly.wc) + (transposed ? k * static_cast<int64_t>(ly.wout) + f : f * static_cast<int64_t>(ly.win) + k)] = Op::cvt(v);
  }
}

// ---- activations (f32; cvnn.hip / cvnn.py:149-210) --------------------------------------------
struct Act {
  // forward: (u, v) -> (ou, ov)
  static __device__ __forceinline__ void fwd(int act, float c, float u, float v, float& ou, float& ov) {
    if (act == SMC_ACT_MODRELU) {
      const float m = sqrtf(u * u + v * v + 1e-9f);
      const float t = m + c;
      const float g = (t > 0.0f ? t : 0.0f) / m;
      ou = g * u;
      ov = g * v;
    } else if (act == SMC_ACT_ZRELU) {
      const bool keep = u >= 0.0f && v >= 0.0f;
      ou = keep ? u : 0.0f;
      ov = keep ? v : 0.0f;
    } else {
      ou = u;
      ov = v;
    }
  }
  // backward: output gradient (gr, gi) at pre-activation (u, v) -> (gu, gv); dc = d loss / d c share
  static __device__ __forceinline__ void bwd(int act, float c, float u, float v, float gr, float gi, float& gu,
                                             float& gv, float& dc) {
    dc = 0.0f;
    if (act == SMC_ACT_MODRELU) {
      const float m = sqrtf(u * u + v * v + 1e-9f);
      if (m + c > 0.0f) {
        dc = (gr * u + gi * v) / m;
        const float g = (m + c) / m;
        const float k = -(gr * u + gi * v) * c / (m * m * m);
        gu = gr * g + k * u;
        gv = gi * g + k * v;
      } else {
        gu = gv = 0.0f;
      }
    } else if (act == SMC_ACT_ZRELU) {
      const bool keep = u >= 0.0f && v >= 0.0f;
      gu = keep ? gr : 0.0f;
      gv = keep ? gi : 0.0f;
    } else {
      gu = gr;
      gv = gi;
    }
  }
};

// Sum over the 16 batch columns of a C tile (lanes c = 0..15 of one row group g), fixed order.
__device__ __forceinline__ float col_sum16(float x) {
  x += __shfl_xor(x, 8, 64);
  x += __shfl_xor(x, 4, 64);
  x += __shfl_xor(x, 2, 64);
  x += __shfl_xor(x, 1, 64);
  return x;
}

// ---- tile GEMM: acc[rt] += A[16 rows at ap][k0, k1) . B[k0, k1)[16 columns of row tile rt at bp] ----
// ap: this lane's A row (+ g KQ), from global memory (L2); bp: this lane's B row (+ g KQ) of row
// tile 0 in LDS, row tiles ldb * 16 elements apart.  The A fragments of up to 8 K blocks are loaded
// before their MFMAs, so their L2 latencies overlap.
template <class Op, int RT>
__device__ __forceinline__ void tile_gemm(f32x4* acc, const typename Op::T* ap, const typename Op::T* bp, int ldb,
                                          int k0, int k1) {
  using V = typename Op::V;
  constexpr int KB = Op::KB;
  for (int kb0 = k0; kb0 < k1; kb0 += 8 * KB) {
    V av[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (kb0 + i * KB < k1) av[i] = Op::ld(ap + kb0 + i * KB);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (kb0 + i * KB < k1) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt] = Op::mmav(acc[rt], av[i], Op::ld(bp + rt * 16 * ldb + kb0 + i * KB));
      }
    }
  }
}

// 512 threads (8 waves, two workgroups per CU at the 4-waves-per-SIMD register budget): beside the path kernel's
// store stream each workgroup's chain of dependent global loads waits microseconds per load, and a second
// workgroup per CU overlaps it (round 5, profiles/r05/bench_fb_threads.txt: lock-step 0.320 -> 0.305 ms/step;
// the network alone on 32 CUs beside an HBM write storm 286 -> 211-236 us; a persistent form with biases and
// weights staged in LDS measured 271 us alone and 0.313-0.315 ms/step and was not kept)
constexpr int kFbThreads = 512;
constexpr int kFbWaves = kFbThreads / 64;

// K split of a layer GEMM with `ntile` output tiles: waves take (tile, K part) items when the
// tiles alone would leave waves idle; parts are added in order 0, 1, ... (bit-reproducible).
__host__ __device__ inline int k_split(int ntile, int kdim, int kb) {
  int ks = 1;
  while (ntile * ks * 2 <= kFbWaves && kdim % (2 * ks * kb) == 0) ks *= 2;
  return ks;
}

// All output tiles of one layer GEMM, then epi(tile, acc) for each; called by every wave.
template <class Op, int RT, class Epi>
__device__ __forceinline__ void layer_gemm(int ntile, int kdim, const typename Op::T* a0, int lda,
                                           const typename Op::T* b0, int ldb, f32x4* scratch, Epi&& epi) {
  constexpr int KQ = Op::KB / 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int ks = k_split(ntile, kdim, Op::KB);
  if (ks == 1) {
    for (int t = wave; t < ntile; t += kFbWaves) {
      f32x4 acc[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      tile_gemm<Op, RT>(acc, a0 + static_cast<int64_t>(t * 16 + c) * lda + g * KQ, b0 + c * ldb + g * KQ, ldb, 0,
                        kdim);
      epi(t, acc);
    }
    return;
  }
  const int kc = kdim / ks;
  const int t = wave / ks, part = wave % ks;
  f32x4 acc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) acc[rt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  if (t < ntile) {
    tile_gemm<Op, RT>(acc, a0 + static_cast<int64_t>(t * 16 + c) * lda + g * KQ, b0 + c * ldb + g * KQ, ldb,
                      part * kc, part * kc + kc);
    if (part > 0) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) scratch[(wave * RT + rt) * 64 + lane] = acc[rt];
    }
  }
  __syncthreads();
  if (t < ntile && part == 0) {
    for (int p = 1; p < ks; ++p) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt] += scratch[((wave + p) * RT + rt) * 64 + lane];
    }
    epi(t, acc);
  }
}

// ---- forward + backward over 16 RT batch rows ------------------------------------------------
template <class Op, int RT>
__global__ __launch_bounds__(kFbThreads) void fb_kernel(MArgs a) {
  using T = typename Op::T;
  constexpr int R = 16 * RT;
  extern __shared__ __attribute__((aligned(16))) char net_lds[];
  __shared__ MLayer layer[kMaxL];
  __shared__ double red[kFbWaves];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, c = lane & 15;
  if (tid < kMaxL) {
#pragma unroll
    for (int i = 0; i < kMaxL; ++i)
      if (i == tid) layer[i] = a.layer[i];
  }
  __syncthreads();
  const int L = a.n_layers;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * R;
  const int64_t bp = a.bp;
  T* ws = static_cast<T*>(a.opws);
  f32x4* scratch = reinterpret_cast<f32x4*>(net_lds);  // [kFbWaves][RT][64] split-K partials
  T* zbuf[2];
  zbuf[0] = reinterpret_cast<T*>(net_lds + kFbWaves * RT * 64 * sizeof(f32x4));
  zbuf[1] = zbuf[0] + R * a.zs;
  T* gb = zbuf[1] + R * a.zs;
  float* pre_lds = reinterpret_cast<float*>(gb + R * a.gs);  // 16-byte aligned: R * gs * sizeof(T) is
  const float* P = a.params;

  // ---- layer-0 input: Z_0 (interleaved re, im) into LDS and Z_0^T (+ ones row) into the workspace
  {
    const MLayer& l0 = layer[0];
    const int n0 = l0.ni;
    auto in = [&](int64_t row, int k) -> float {
      if (row >= a.batch || k >= 2 * n0) return 0.0f;
      const int64_t i = row * n0 + (k >> 1);
      return (k & 1) ? (a.in_im ? a.in_im[i] : 0.0f) : a.in_re[i];
    };
    for (int i = tid; i < R * l0.win; i += kFbThreads) {
      const int r = i / l0.win, k = i - r * l0.win;
      zbuf[0][r * a.zs + k] = Op::cvt(in(r0 + r, k));
    }
    for (int i = tid; i < l0.kx * R; i += kFbThreads) {
      const int k = i / R, r = i - k * R;
      ws[l0.zt + k * bp + r0 + r] = Op::cvt(k == 2 * n0 ? 1.0f : in(r0 + r, k));
    }
  }
  __syncthreads();

  // ---- forward through the hidden layers
  int cur = 0;
  for (int l = 0; l + 1 < L; ++l) {
    const MLayer& ly = layer[l];
    const MLayer& nx = layer[l + 1];
    T* zout = zbuf[cur ^ 1];
    layer_gemm<Op, RT>(ly.wout / 16, ly.win, ws + ly.wc, ly.win, zbuf[cur], a.zs, scratch, [&](int ft, f32x4* acc) {
      const int f0 = ft * 16 + 4 * g;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int r = rt * 16 + c;
        float o[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = (f0 >> 1) + h;
          o[2 * h] = o[2 * h + 1] = 0.0f;
          if (j < ly.no) {
            float u = acc[rt][2 * h], v = acc[rt][2 * h + 1];
            if (ly.b_re >= 0) u += P[ly.b_re + j];
            if (ly.b_im >= 0) v += P[ly.b_im + j];
            if (ly.pre >= 0) {
              float* pre = (a.pre_global ? a.fws + r0 * (2 * ly.no) : pre_lds) + ly.pre + r * (2 * ly.no) + 2 * j;
              pre[0] = u;
              pre[1] = v;
            }
            Act::fwd(ly.act, ly.act == SMC_ACT_MODRELU ? P[ly.act_bias + j] : 0.0f, u, v, o[2 * h], o[2 * h + 1]);
          }
        }
        Op::store4(zout + r * a.zs + f0, o[0], o[1], o[2], o[3]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (f0 + i < 2 * ly.no) ws[nx.zt + (f0 + i) * bp + r0 + r] = Op::cvt(o[i]);
      }
    });
    // Z^T rows 2 no .. kx of the next layer: the ones row, then zeros
    for (int i = tid; i < (nx.kx - 2 * ly.no) * R; i += kFbThreads) {
      const int k = 2 * ly.no + i / R, r = i % R;
      ws[nx.zt + k * bp + r0 + r] = Op::cvt(k == 2 * ly.no ? 1.0f : 0.0f);
    }
    __syncthreads();
    cur ^= 1;
  }

  // ---- last layer: prediction, loss, output gradient (+ its activation backward) into gb / dU^T
  const float scale = 2.0f / static_cast<float>(static_cast<double>(a.batch) * layer[L - 1].no);
  double loss = 0.0;
  {
    const MLayer& ly = layer[L - 1];
    const int N = ly.no;
    layer_gemm<Op, RT>(ly.wout / 16, ly.win, ws + ly.wc, ly.win, zbuf[cur], a.zs, scratch, [&](int ft, f32x4* acc) {
      const int f0 = ft * 16 + 4 * g;
      float dcs[2] = {0.0f, 0.0f};
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int r = rt * 16 + c;
        const int64_t row = r0 + r;
        float o[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = (f0 >> 1) + h;
          o[2 * h] = o[2 * h + 1] = 0.0f;
          if (j < N && row < a.batch) {
            float u = acc[rt][2 * h], v = acc[rt][2 * h + 1];
            if (ly.b_re >= 0) u += P[ly.b_re + j];
            if (ly.b_im >= 0) v += P[ly.b_im + j];
            const float cb = ly.act == SMC_ACT_MODRELU ? P[ly.act_bias + j] : 0.0f;
            float pr, pi;
            Act::fwd(ly.act, cb, u, v, pr, pi);
            const float* t = a.targets + (row * N + j) * 2;
            const float dr = pr - t[0], di = pi - t[1];
            loss += static_cast<double>(dr * dr) + static_cast<double>(di * di);
            float dc;
            Act::bwd(ly.act, cb, u, v, scale * dr, scale * di, o[2 * h], o[2 * h + 1], dc);
            dcs[h] += dc;
          }
        }
        Op::store4(gb + r * a.gs + f0, o[0], o[1], o[2], o[3]);
#pragma unroll
        for (int i = 0; i < 4; ++i) ws[ly.gt + (f0 + i) * bp + r0 + r] = Op::cvt(o[i]);
      }
      if (ly.cpart >= 0) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float s = col_sum16(dcs[h]);
          const int j = (f0 >> 1) + h;
          if (c == 0 && j < N) a.fws[ly.cpart + static_cast<int64_t>(blockIdx.x) * N + j] = s;
        }
      }
    });
  }
  // workgroup loss partial, fixed order: wave butterfly, then waves in order
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) loss += __shfl_xor(loss, off, 64);
  if (lane == 0) red[wave] = loss;
  __syncthreads();  // also: gb complete, split-K scratch free
  if (tid == 0) {
    double t = 0.0;
    for (int w = 0; w < kFbWaves; ++w) t += red[w];
    a.lossp[blockIdx.x] = t;
  }

  // ---- input gradients down the layers: dZ_l = dU_l Wc_l, then layer l-1's activation backward
  const T* gsrc = gb;
  int gstride = a.gs;
  int dst = 0;
  for (int l = L - 1; l >= 1; --l) {
    const MLayer& ly = layer[l];
    const MLayer& lp = layer[l - 1];
    T* gdst = zbuf[dst];
    layer_gemm<Op, RT>(ly.win / 16, ly.wout, ws + ly.wct, ly.wout, gsrc, gstride, scratch, [&](int it, f32x4* acc) {
      const int f0 = it * 16 + 4 * g;
      float dcs[2] = {0.0f, 0.0f};
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int r = rt * 16 + c;
        float o[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = (f0 >> 1) + h;
          o[2 * h] = o[2 * h + 1] = 0.0f;
          if (j < lp.no) {
            float u = 0.0f, v = 0.0f;
            if (lp.pre >= 0) {
              const float* pre =
                  (a.pre_global ? a.fws + r0 * (2 * lp.no) : pre_lds) + lp.pre + r * (2 * lp.no) + 2 * j;
              u = pre[0];
              v = pre[1];
            }
            const float cb = lp.act == SMC_ACT_MODRELU ? P[lp.act_bias + j] : 0.0f;
            float dc;
            Act::bwd(lp.act, cb, u, v, acc[rt][2 * h], acc[rt][2 * h + 1], o[2 * h], o[2 * h + 1], dc);
            dcs[h] += dc;
          }
        }
        Op::store4(gdst + r * a.zs + f0, o[0], o[1], o[2], o[3]);
#pragma unroll
        for (int i = 0; i < 4; ++i) ws[lp.gt + (f0 + i) * bp + r0 + r] = Op::cvt(o[i]);
      }
      if (lp.cpart >= 0) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float s = col_sum16(dcs[h]);
          const int j = (f0 >> 1) + h;
          if (c == 0 && j < lp.no) a.fws[lp.cpart + static_cast<int64_t>(blockIdx.x) * lp.no + j] = s;
        }
      }
    });
    __syncthreads();
    gsrc = gdst;
    gstride = a.zs;
    dst ^= 1;
  }
}

// ---- weight gradients: one workgroup per (layer, 64 features, 64 columns, batch segment) ------
// dWc block [64 f][64 k] = sum over the segment's rows of dU^T[f][row] Z^T[k][row]: both operands
// staged through LDS in 64-row K stages (double-buffered, the next stage's global loads in flight
// during the current stage's MFMAs); wave w computes the 32 x 32 quarter (w / 2, w % 2) as 2 x 2
// tiles.  Workgroups past the tile blocks sum the loss and modReLU-bias partials of one segment
// per wave.
// Bookkeeping items of the weight-gradient launch: wave w of bookkeeping workgroup `item` sums the
// loss and modReLU-bias partials of batch segment 4 item + w into that segment's partials row.
__device__ void wgrad_bookkeeping(const MArgs& a, int64_t item, int wave, int lane) {
  const int64_t sg = item * kWaves + wave;
  if (sg >= a.segs) return;
  const int s = static_cast<int>(sg);
  const int64_t seg_rows = a.bp / a.segs;
  const int w0 = static_cast<int>(s * (seg_rows / a.rows)), w1 = static_cast<int>((s + 1) * (seg_rows / a.rows));
  float* part = a.partials + s * (a.n_params + 1);
  if (lane == 0) {
    double t = 0.0;
    for (int w = w0 * a.lpb; w < w1 * a.lpb; ++w) t += a.lossp[w];
    part[a.n_params] = static_cast<float>(t / (static_cast<double>(a.batch) * a.layer[a.n_layers - 1].no));
  }
  for (int ll = 0; ll < a.n_layers; ++ll) {
    const MLayer& ly = a.layer[ll];
    if (ly.cpart < 0) continue;
    for (int j = lane; j < ly.no; j += 64) {
      double t = 0.0;
      for (int w = w0; w < w1; ++w) t += a.fws[ly.cpart + static_cast<int64_t>(w) * ly.no + j];
      part[ly.act_bias + j] = static_cast<float>(t);
    }
  }
}

// (settled values; tools/micro/make_variant.py edits these lines for A/B builds)
constexpr bool kWgradRowMajor = true;  // layered plans: wgrad reads Z_l / dU_l row-major, lgemm writes no ^T copies
// f32 batch rows per K stage: 16 (20 KiB of LDS, 8 workgroups per CU) runs C2/H = 256's 1216 weight-
// gradient items in one round where 32 (36 KiB, 4 per CU) left a second round of 192 (round-4 A/B:
// isolated H = 256 network 251-253 -> 243 us, profiles/r04/ab_wgrad_stage.txt)
constexpr int kWgradKsF32 = 16;
constexpr int kWgBlock = 64;  // output block edge
constexpr int kWgStage = 64;  // batch rows per K stage (bf16; 32 for f32: the same 36 KiB of LDS)

// the weight-gradient block's partials (dA, dB, biases) of segment s from the accumulators
__device__ __forceinline__ void wgrad_store(const MArgs& a, const MLayer& ly, int s, int64_t stride, int f_base,
                                            int k_base, int wm, int wn, int g, int c, const f32x4 (&acc)[2][2]) {
  float* part = a.partials + s * stride;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int fbase = f_base + wm * 32 + i * 16 + 4 * g;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      float y[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = __shfl_xor(acc[i][jt][r], 1, 64);
      const int k = k_base + wn * 32 + jt * 16 + c;
      if ((c & 1) == 0 && k < ly.kx) {
        const int kk = k >> 1;
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const int j = (fbase + r) >> 1;
          if (j >= ly.no) continue;
          if (kk < ly.ni) {
            const int64_t w = static_cast<int64_t>(j) * ly.ni + kk;
            part[ly.w_re + w] = acc[i][jt][r] + y[r + 1];
            part[ly.w_im + w] = acc[i][jt][r + 1] - y[r];
          } else if (kk == ly.ni) {  // the ones column: bias gradients
            if (ly.b_re >= 0) part[ly.b_re + j] = acc[i][jt][r];
            if (ly.b_im >= 0) part[ly.b_im + j] = acc[i][jt][r + 1];
          }
        }
      }
    }
  }
}

template <class Op>
__global__ __launch_bounds__(kThreads) void wgrad_kernel(MArgs a) {
  using T = typename Op::T;
  using V = typename Op::V;
  constexpr int KB = Op::KB, KQ = KB / 4;
  constexpr int ES = static_cast<int>(sizeof(T));
  constexpr int KS = ES == 2 ? kWgStage : kWgradKsF32;  // batch rows per K stage
  constexpr int LD = KS + 16 / ES;                       // LDS row stride (elements): odd multiple of 16 B
  constexpr int PER = kWgBlock * KS / kThreads;          // elements each thread stages per operand
  constexpr int NV = PER * ES / 16;                   // 16-byte loads per operand per thread
  __shared__ __attribute__((aligned(16))) T stage[2][2][kWgBlock * LD];  // [buffer][A, B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, c = lane & 15;
  const T* ws = static_cast<const T*>(a.opws);
  const int64_t stride = a.n_params + 1;
  const int64_t seg_rows = a.bp / a.segs;
  int64_t item = blockIdx.x;
  int l = 0;
  while (l < a.n_layers && item >= a.layer[l].items) item -= a.layer[l].items, ++l;
  if (l == a.n_layers) {
    wgrad_bookkeeping(a, item, wave, lane);
    return;
  }
  const MLayer& ly = a.layer[l];
  const int nfb = (ly.wout + kWgBlock - 1) / kWgBlock, nkb = (ly.kx + kWgBlock - 1) / kWgBlock;
  const int s = static_cast<int>(item % a.segs);
  const int64_t rest = item / a.segs;
  const int kblk = static_cast<int>(rest % nkb);
  const int fblk = static_cast<int>(rest / nkb);
  (void)nfb;
  const int f_base = fblk * kWgBlock, k_base = kblk * kWgBlock;
  const int64_t b0 = s * seg_rows;
  // staging map: thread -> row tid / 4 of the block, elements (tid % 4) * 16 .. + 16 of the stage
  const int srow = tid >> 2, scol = (tid & 3) * PER;
  const bool a_ok = f_base + srow < ly.wout, b_ok = k_base + srow < ly.kx;
  const T* ag = ws + ly.gt + (f_base + srow) * a.bp + b0 + scol;
  const T* bg = ws + ly.zt + (k_base + srow) * a.bp + b0 + scol;
  typedef float raw4 __attribute__((ext_vector_type(4)));
  raw4 ra[NV], rb[NV];
  auto fetch = [&](int64_t kb) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      ra[v] = a_ok ? *reinterpret_cast<const raw4*>(ag + kb + v * (16 / ES)) : raw4{0.f, 0.f, 0.f, 0.f};
      rb[v] = b_ok ? *reinterpret_cast<const raw4*>(bg + kb + v * (16 / ES)) : raw4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto put = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      *reinterpret_cast<raw4*>(&stage[buf][0][srow * LD + scol + v * (16 / ES)]) = ra[v];
      *reinterpret_cast<raw4*>(&stage[buf][1][srow * LD + scol + v * (16 / ES)]) = rb[v];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const int wm = wave >> 1, wn = wave & 1;
  const int nst = static_cast<int>(seg_rows / KS);
  fetch(0);
  put(0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) fetch(static_cast<int64_t>(st + 1) * KS);
#pragma unroll
    for (int kb = 0; kb < KS; kb += KB) {
      V af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = Op::ld(&stage[buf][0][(wm * 32 + i * 16 + c) * LD + kb + g * KQ]);
        bf[i] = Op::ld(&stage[buf][1][(wn * 32 + i * 16 + c) * LD + kb + g * KQ]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = Op::mmav(acc[i][j], af[i], bf[j]);
    }
    if (st + 1 < nst) put(buf ^ 1);
    __syncthreads();
  }
  wgrad_store(a, ly, s, stride, f_base, k_base, wm, wn, g, c, acc);
}

// wgrad for layered plans (round 4): the operands straight from the row-major Z_l [bp][kx] and
// dU_l [bp][wout] the layered GEMMs write anyway, so their epilogues store no ^T copies.  Each K stage
// stages KS batch rows x 64 features of both operands (16-B loads along the features, the row stride
// 68 floats: lanes c and the 4 row groups g hit distinct banks); a lane's MFMA operand k-values are the
// 4 batch rows 4 g .. 4 g + 3 of the block -- the same (row, MFMA) assignment as wgrad_kernel's
// transposed fragments, so the partials are bit-identical to it.
template <int KS>
__global__ __launch_bounds__(kThreads) void wgrad_rm_kernel(MArgs a) {
  constexpr int LD = kWgBlock + 4;  // 4 LD = 16 (mod 64): the 4 row groups g read distinct banks
  constexpr int NV = KS * kWgBlock / 4 / kThreads;  // 16-B loads per operand per thread and stage
  static_assert(NV >= 1 && KS % 16 == 0, "whole 16-row MFMA blocks per stage");
  __shared__ __attribute__((aligned(16))) float stage[2][2][KS * LD];  // [buffer][A = dU, B = Z]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, c = lane & 15;
  const float* ws = static_cast<const float*>(a.opws);
  const int64_t stride = a.n_params + 1;
  const int64_t seg_rows = a.bp / a.segs;
  int64_t item = blockIdx.x;
  int l = 0;
  while (l < a.n_layers && item >= a.layer[l].items) item -= a.layer[l].items, ++l;
  if (l == a.n_layers) {
    wgrad_bookkeeping(a, item, wave, lane);
    return;
  }
  const MLayer& ly = a.layer[l];
  const int nkb = (ly.kx + kWgBlock - 1) / kWgBlock;
  const int s = static_cast<int>(item % a.segs);
  const int64_t rest = item / a.segs;
  const int kblk = static_cast<int>(rest % nkb);
  const int fblk = static_cast<int>(rest / nkb);
  const int f_base = fblk * kWgBlock, k_base = kblk * kWgBlock;
  const int64_t b0 = s * seg_rows;
  const float* G = ws + ly.dr;  // [bp][wout]
  const float* Z = ws + ly.zr;  // [bp][kx]
  f32x4 ra[NV], rb[NV];
  auto fetch = [&](int64_t kb) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = v * kThreads + tid, r = i / (kWgBlock / 4), q = 4 * (i % (kWgBlock / 4));
      const int64_t row = b0 + kb + r;
      const bool oa = f_base + q < ly.wout, ob = k_base + q < ly.kx;
      const f32x4 x = *reinterpret_cast<const f32x4*>(G + (oa ? row * ly.wout + f_base + q : 0));
      const f32x4 y = *reinterpret_cast<const f32x4*>(Z + (ob ? row * ly.kx + k_base + q : 0));
      ra[v] = oa ? x : f32x4{0.f, 0.f, 0.f, 0.f};
      rb[v] = ob ? y : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto put = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = v * kThreads + tid, r = i / (kWgBlock / 4), q = 4 * (i % (kWgBlock / 4));
      *reinterpret_cast<f32x4*>(&stage[buf][0][r * LD + q]) = ra[v];
      *reinterpret_cast<f32x4*>(&stage[buf][1][r * LD + q]) = rb[v];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  const int wm = wave >> 1, wn = wave & 1;
  const int nst = static_cast<int>(seg_rows / KS);
  fetch(0);
  put(0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) fetch(static_cast<int64_t>(st + 1) * KS);
#pragma unroll
    for (int kb = 0; kb < KS; kb += 16) {
      f32x4 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          af[i][r] = stage[buf][0][(kb + 4 * g + r) * LD + wm * 32 + i * 16 + c];
          bf[i][r] = stage[buf][1][(kb + 4 * g + r) * LD + wn * 32 + i * 16 + c];
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = OpF32::mmav(acc[i][j], af[i], bf[j]);
    }
    if (st + 1 < nst) put(buf ^ 1);
    __syncthreads();
  }
  wgrad_store(a, ly, s, stride, f_base, k_base, wm, wn, g, c, acc);
}

// ---- layered step for wide layers (round 3) ----------------------------------------------------
// fb_kernel keeps 16 batch rows on chip through every layer, so each of its workgroups streams every
// weight matrix from L2: at H = 256 (1 MB per hidden layer) that is ~1 GB of L2 reads per step and the
// step ran at 0.26 of the f32 MFMA peak.  Wide networks instead run one GEMM launch per layer and
// direction over 128-feature x 64-row tiles, both operands staged through LDS in 64-deep K stages
// (double-buffered, the next stage's global loads and the next 16-deep block's LDS fragments in flight
// during the MFMAs; tools/micro/lgemm.hip: 0.55 of the f32 peak on the 512 x 4096 x 512 GEMM), with
// the bias as an extra weight column against Z's ones column and the epilogues of fb_kernel fused:
//   kLFwd  (hidden layer l): pre-activations -> workspace, activation -> Z_{l+1} (row-major and ^T)
//   kLLast (last layer): prediction, loss partial, output gradient -> dU_L (row-major and ^T)
//   kLBwd  (layer l, l >= 1): dZ_l = dU_l Wc_l, layer l-1's activation backward -> dU_{l-1}
// wgrad_kernel then reads the ^T copies exactly as after fb_kernel (same partials, same reduction).
// LDS row stride kLK + 8 floats: a ds_read_b128 fragment (lane 16 g + c: row c, 16 B at 16 g) is serviced in
// four 16-lane groups ({0-3, 12-15, 20-27}, ...; MI355X_MICROARCH.md, LDS), and at stride 68 every group
// had two lanes on one bank quad (PMC: 1.4e6 conflict cycles per H = 256 GEMM); 72 is conflict-free
constexpr int kLM = 64, kLN = 64, kLK = 64, kLLd = kLK + 8;  // tile (features x batch rows), K stage, LDS stride
// waves: 4 along the features (kLM / 4 each) x kLWR along the batch rows (kLN / kLWR each); kLM = 64: 512
// workgroups at H = 256 (263 vs 269 us per step with 128).  8 waves (2 row groups): 4 waves per SIMD at two
// workgroups per CU, the isolated H = 256 network 237-240 -> 228-230 us against 4 waves
// (profiles/r04/net/ab_lgemm_waves.txt)
constexpr int kLThreads = 512;
constexpr int kLWF = 4, kLWR = kLThreads / 64 / kLWF;
constexpr int kLTM = kLM / kLWF / 16, kLTN = kLN / kLWR / 16;  // 16 x 16 tiles per wave
enum { kLFwd = 0, kLLast = 1, kLBwd = 2 };

// Wc [wout][kx] with the bias column, Wc^T [win][wout], and Z_0 / Z_0^T from the inputs (+ ones
// column): blockIdx.y = region (2 l: Wc_l, 2 l + 1: Wc_l^T, 2 L: Z_0, 2 L + 1: Z_0^T), a grid-stride
// loop over the region's rows and columns
__global__ __launch_bounds__(kThreads) void lpack_kernel(MArgs a) {
  float* ws = static_cast<float*>(a.opws);
  const int reg = blockIdx.y;
  const int L = a.n_layers;
  if (reg < 2 * L) {
    const MLayer& ly = a.layer[reg >> 1];
    const bool transposed = reg & 1;
    const int rows = transposed ? ly.win : ly.wout, cols = transposed ? ly.wout : ly.kx;
    for (int64_t e = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; e < static_cast<int64_t>(rows) * cols;
         e += static_cast<int64_t>(gridDim.x) * kThreads) {
      const int rr = static_cast<int>(e / cols), cc = static_cast<int>(e % cols);
      const int f = transposed ? cc : rr, k = transposed ? rr : cc;
      const int j = f >> 1, kk = k >> 1, ra = f & 1, rb = k & 1;
      float v = 0.0f;
      if (j < ly.no && kk < ly.ni) {
        const float wa = a.params[ly.w_re + static_cast<int64_t>(j) * ly.ni + kk];
        const float wb = a.params[ly.w_im + static_cast<int64_t>(j) * ly.ni + kk];
        v = ra == rb ? wa : (ra == 0 ? -wb : wb);
      } else if (j < ly.no && !transposed && k == 2 * ly.ni) {  // bias column: (b_re, b_im) of output j
        const int64_t bo = ra == 0 ? ly.b_re : ly.b_im;
        v = bo >= 0 ? a.params[bo + j] : 0.0f;
      }
      ws[(transposed ? ly.wct : ly.wc) + e] = v;
    }
    return;
  }
  // Z_0 [bp][kx] and Z_0^T [kx][bp]: interleaved (re, im) inputs, the ones column at 2 ni, zeros
  const MLayer& l0 = a.layer[0];
  const bool transposed = reg == 2 * L + 1;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; e < a.bp * l0.kx;
       e += static_cast<int64_t>(gridDim.x) * kThreads) {
    const int64_t row = transposed ? e % a.bp : e / l0.kx;
    const int k = static_cast<int>(transposed ? e / a.bp : e % l0.kx);
    float v = k == 2 * l0.ni ? 1.0f : 0.0f;
    if (k < 2 * l0.ni && row < a.batch) {
      const int64_t i = row * l0.ni + (k >> 1);
      v = (k & 1) ? (a.in_im ? a.in_im[i] : 0.0f) : a.in_re[i];
    }
    ws[(transposed ? l0.zt : l0.zr) + e] = v;
  }
}

// XCD-aware tile order: the 1-D grid's consecutive workgroups go round-robin to the 8 XCDs, so
// workgroup w runs on XCD w % 8; each XCD takes a contiguous eighth of the batch blocks with every
// feature block, and reads only its eighth of the row operand (B) and the whole weight matrix (A)
// into its own L2, instead of every XCD streaming all of B past one feature block
// (NB not a multiple of 8: the grid is rounded up to 8 equal XCD ranges and the workgroups past the
// last batch block return at once).  False: this workgroup has no tile.
__device__ __forceinline__ bool lgemm_tile(const MArgs& a, int& mb, int& nb) {
  const int MB = static_cast<int>(a.lgemm_mb);
  const int NB = static_cast<int>(a.bp / kLN);
  const int per = (NB + 7) >> 3;
  const int xcd = static_cast<int>(blockIdx.x) & 7, local = static_cast<int>(blockIdx.x) >> 3;
  nb = xcd * per + local / MB;
  mb = local % MB;
  return nb < NB;
}

// the epilogue's global inputs (targets / pre-activations) of this thread's rows, loaded before the K
// loop so that their latency hides behind it: two waves per SIMD cannot hide a load latency per row
constexpr int kLRows = kLN / (kLThreads / (kLM / 4));  // epilogue rows per thread (4)
template <int MODE>
__device__ __forceinline__ void lgemm_prefetch(const MArgs& a, int l, int m0, int64_t n0, float2 (&in)[kLRows][2]) {
  const int tid = threadIdx.x;
  const MLayer& lo = MODE == kLBwd ? a.layer[l - 1] : a.layer[l];
  const int N = lo.no;
  const int q = tid % (kLM / 4), rb0 = tid / (kLM / 4);
  const int f0 = m0 + 4 * q;
#pragma unroll
  for (int k = 0; k < kLRows; ++k) {
    const int64_t b = n0 + rb0 + k * (kLThreads / (kLM / 4));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int jj = (f0 >> 1) + h;
      in[k][h] = float2{0.0f, 0.0f};
      if (MODE == kLLast && jj < N && b < a.batch) in[k][h] = *reinterpret_cast<const float2*>(a.targets + (b * N + jj) * 2);
      if (MODE == kLBwd && jj < N && lo.pre >= 0) in[k][h] = *reinterpret_cast<const float2*>(a.fws + lo.pre + b * (2 * N) + 2 * jj);
    }
  }
}

// ---- epilogue, from the [row][feature] tile of the accumulators in LDS (written and synchronised by
// the caller): each thread takes 4 features of one batch row (row-major outputs, 16-B stores along the
// features) and finally, without kWgradRowMajor, whole 64-row feature lines (the ^T copies, 16-B
// stores along the batch): every global store is a full 16-B piece of a contiguous line
constexpr int kLTld = kLM + 4;  // tile row stride (floats): [row][feature], 16-B pieces conflict-free
template <int MODE>
__device__ __forceinline__ void lgemm_epilogue(const MArgs& a, int l, int mb, int nb, float* tile, float* part,
                                               double* red, const float2 (&in)[kLRows][2]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* ws = static_cast<float*>(a.opws);
  const float* P = a.params;
  const MLayer& ly = a.layer[l];
  const MLayer& lo = MODE == kLBwd ? a.layer[l - 1] : ly;  // the layer whose output (gradient) this launch writes
  const int N = lo.no;
  const int MB = static_cast<int>(a.lgemm_mb);
  const int m0 = mb * kLM;
  const int64_t n0 = static_cast<int64_t>(nb) * kLN;
  const int q = tid % (kLM / 4), rb0 = tid / (kLM / 4);
  const int f0 = m0 + 4 * q;
  const int64_t bp = a.bp;
  const int64_t blk = nb;  // batch block of kLN rows (= a.rows)
  // the layer whose output (or output gradient) this launch writes, and its row-major / ^T buffers
  const MLayer& nx = MODE == kLFwd ? a.layer[l + 1] : ly;
  const int64_t rm_off = MODE == kLFwd ? nx.zr : lo.dr;
  const int64_t tr_off = MODE == kLFwd ? nx.zt : lo.gt;
  const int rm_ld = MODE == kLFwd ? nx.kx : lo.wout;  // row-major row length
  const int nvalid = MODE == kLFwd ? ly.wout : lo.wout;  // features this launch writes
  const float scale = 2.0f / static_cast<float>(static_cast<double>(a.batch) * ly.no);
  double loss = 0.0;
  float dcs[2] = {0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < kLRows; ++k) {
    const int rr = rb0 + k * (kLThreads / (kLM / 4));
    const int64_t b = n0 + rr;
    const f32x4 x = *reinterpret_cast<const f32x4*>(&tile[rr * kLTld + 4 * q]);
    float o[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int jj = (f0 >> 1) + h;
      const float u = x[2 * h], v = x[2 * h + 1];
      o[2 * h] = o[2 * h + 1] = 0.0f;
      if constexpr (MODE == kLFwd) {
        if (jj < ly.no) {
          if (ly.pre >= 0) *reinterpret_cast<float2*>(a.fws + ly.pre + b * (2 * ly.no) + 2 * jj) = float2{u, v};
          Act::fwd(ly.act, ly.act == SMC_ACT_MODRELU ? P[ly.act_bias + jj] : 0.0f, u, v, o[2 * h], o[2 * h + 1]);
        } else {
          o[2 * h] = 2 * jj == 2 * ly.no ? 1.0f : 0.0f;  // Z_{l+1}'s ones column, then zeros
        }
      } else if (jj < N && (MODE == kLBwd || b < a.batch)) {
        const float cb = lo.act == SMC_ACT_MODRELU ? P[lo.act_bias + jj] : 0.0f;
        float dc;
        if constexpr (MODE == kLLast) {
          float pr, pi;
          Act::fwd(lo.act, cb, u, v, pr, pi);
          const float2 t = in[k][h];
          const float dr = pr - t.x, di = pi - t.y;
          loss += static_cast<double>(dr * dr) + static_cast<double>(di * di);
          Act::bwd(lo.act, cb, u, v, scale * dr, scale * di, o[2 * h], o[2 * h + 1], dc);
        } else {
          const float2 pre = in[k][h];
          Act::bwd(lo.act, cb, pre.x, pre.y, u, v, o[2 * h], o[2 * h + 1], dc);
        }
        dcs[h] += dc;
      }
    }
    if (f0 < nvalid) *reinterpret_cast<f32x4*>(ws + rm_off + b * rm_ld + f0) = f32x4{o[0], o[1], o[2], o[3]};
    if constexpr (!kWgradRowMajor)
      *reinterpret_cast<f32x4*>(&tile[rr * kLTld + 4 * q]) = f32x4{o[0], o[1], o[2], o[3]};  // the ^T copy's values
  }
  if constexpr (MODE != kLFwd) {
    // modReLU bias share of the block's kLN rows: each thread's rows in order, then the kLN / 8 row
    // groups in order (through LDS, after the ^T tile is complete)
    if (lo.cpart >= 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h) part[rb0 * (kLM / 2) + 2 * q + h] = dcs[h];
    }
    if constexpr (MODE == kLLast) {  // block loss partial: thread sums, wave butterfly, waves in order
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) loss += __shfl_xor(loss, off, 64);
      if (lane == 0) red[wave] = loss;
    }
    __syncthreads();
    if (lo.cpart >= 0 && tid < kLM / 2) {
      const int jj = m0 / 2 + tid;
      float s = 0.0f;
      for (int w = 0; w < kLThreads / (kLM / 4); ++w) s += part[w * (kLM / 2) + tid];
      if (jj < N) a.fws[lo.cpart + blk * N + jj] = s;
    }
    if (MODE == kLLast && tid == 0) {
      double t = 0.0;
      for (int w = 0; w < kLThreads / 64; ++w) t += red[w];
      a.lossp[blk * a.lpb + mb] = t;
    }
  } else {
    __syncthreads();
  }
  // phase C: the ^T copy, whole 64-row lines of each feature (only for the transposed wgrad_kernel)
  for (int e = tid; e < (kWgradRowMajor ? 0 : kLM * (kLN / 4)); e += kLThreads) {
    const int fr = e / (kLN / 4), q4 = e % (kLN / 4);
    if (m0 + fr < nvalid)
      *reinterpret_cast<f32x4*>(ws + tr_off + static_cast<int64_t>(m0 + fr) * bp + n0 + 4 * q4) =
          f32x4{tile[(4 * q4) * kLTld + fr], tile[(4 * q4 + 1) * kLTld + fr], tile[(4 * q4 + 2) * kLTld + fr],
                tile[(4 * q4 + 3) * kLTld + fr]};
  }
  if constexpr (MODE == kLFwd) {
    // columns [wout, kx_{l+1}) of Z_{l+1} (the ones column when 2 no is a multiple of 16)
    if (mb == MB - 1) {
      for (int e = tid; e < (nx.kx - ly.wout) * kLN; e += kLThreads) {
        const int k = ly.wout + e / kLN;
        const int64_t b = n0 + e % kLN;
        const float v = k == 2 * ly.no ? 1.0f : 0.0f;
        ws[nx.zr + b * nx.kx + k] = v;
        if constexpr (!kWgradRowMajor) ws[nx.zt + static_cast<int64_t>(k) * bp + b] = v;
      }
    }
  }
}

// C[m][n] = sum_k A[m][k] B[n][k]: fwd / last A = Wc [wout][kx], B = Z_l [bp][kx];
// bwd A = Wc^T [win][wout], B = dU_l [bp][wout]
struct LOperands {
  const float* A;
  const float* B;
  int K, Mrows;
};
template <int MODE>
__device__ __forceinline__ LOperands lgemm_operands(const MArgs& a, int l) {
  const MLayer& ly = a.layer[l];
  const bool bwd = MODE == kLBwd;
  const float* ws = static_cast<const float*>(a.opws);
  return LOperands{ws + (bwd ? ly.wct : ly.wc), ws + (bwd ? ly.dr : ly.zr), bwd ? ly.wout : ly.kx,
                   bwd ? ly.win : ly.wout};
}

template <int MODE>
__global__ __launch_bounds__(kLThreads) void lgemm_kernel(MArgs a, int l) {
  __shared__ __attribute__((aligned(16))) float sa[2][kLM * kLLd];
  __shared__ __attribute__((aligned(16))) float sb[2][kLN * kLLd];
  __shared__ double red[kLThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, c = lane & 15;
  const int wf = wave % kLWF, wr = wave / kLWF;  // the wave's feature group and row group
  int mb, nb;
  if (!lgemm_tile(a, mb, nb)) return;  // uniform, before any barrier
  const LOperands op = lgemm_operands<MODE>(a, l);
  const float* A = op.A;
  const float* B = op.B;
  const int K = op.K, Mrows = op.Mrows;
  const int64_t lda = K, ldb = K;
  const int64_t Nrows = a.bp;
  const int m0 = mb * kLM;
  const int64_t n0 = static_cast<int64_t>(nb) * kLN;
  constexpr int AV = kLM * kLK / 4 / kLThreads, BV = kLN * kLK / 4 / kLThreads;
  f32x4 ra[AV], rb[BV];
  // every load is issued (out-of-range pieces read element 0 and are zeroed by a select): a guarded
  // load compiles to a branch around it, eight per stage
  auto fetch = [&](int k0) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int i = v * kLThreads + tid, r = i / (kLK / 4), q = i % (kLK / 4);
      const bool ok = m0 + r < Mrows && k0 + 4 * q < K;
      const f32x4 x = *reinterpret_cast<const f32x4*>(A + (ok ? static_cast<int64_t>(m0 + r) * lda + k0 + 4 * q : 0));
      ra[v] = ok ? x : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int i = v * kLThreads + tid, r = i / (kLK / 4), q = i % (kLK / 4);
      const bool ok = n0 + r < Nrows && k0 + 4 * q < K;
      const f32x4 x = *reinterpret_cast<const f32x4*>(B + (ok ? (n0 + r) * ldb + k0 + 4 * q : 0));
      rb[v] = ok ? x : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto put = [&](int buf) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int i = v * kLThreads + tid, r = i / (kLK / 4), q = i % (kLK / 4);
      *reinterpret_cast<f32x4*>(&sa[buf][r * kLLd + 4 * q]) = ra[v];
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int i = v * kLThreads + tid, r = i / (kLK / 4), q = i % (kLK / 4);
      *reinterpret_cast<f32x4*>(&sb[buf][r * kLLd + 4 * q]) = rb[v];
    }
  };
  float2 in[kLRows][2];
  lgemm_prefetch<MODE>(a, l, m0, n0, in);
  f32x4 acc[kLTM][kLTN];
#pragma unroll
  for (int i = 0; i < kLTM; ++i)
#pragma unroll
    for (int j = 0; j < kLTN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // full K stages run their kLK / 16 blocks unconditionally; the last, partial stage (K a multiple of 16)
  // its remaining blocks: no per-block branch around the MFMAs (each made the accumulators round-trip
  // through VGPRs at the join)
  const int nfull = K / kLK, tail = (K % kLK) / 16;
  const int nst = nfull + (tail ? 1 : 0);
  f32x4 af[2][kLTM], bf[2][kLTN];
  auto ld = [&](int buf, int s, int kb) {
#pragma unroll
    for (int i = 0; i < kLTM; ++i)
      af[s][i] = *reinterpret_cast<const f32x4*>(&sa[buf][((wf * kLTM + i) * 16 + c) * kLLd + kb + 4 * g]);
#pragma unroll
    for (int j = 0; j < kLTN; ++j)
      bf[s][j] = *reinterpret_cast<const f32x4*>(&sb[buf][((wr * kLTN + j) * 16 + c) * kLLd + kb + 4 * g]);
  };
  auto mma = [&](int s) {
#pragma unroll
    for (int i = 0; i < kLTM; ++i)
#pragma unroll
      for (int j = 0; j < kLTN; ++j) acc[i][j] = OpF32::mmav(acc[i][j], af[s][i], bf[s][j]);
  };
  fetch(0);
  put(0);
  __syncthreads();
  // the full K stages: the kLK / 16 blocks unconditionally (no branch around the MFMAs, whose join made
  // the accumulators round-trip through VGPRs); the next stage's loads in flight meanwhile
  for (int st = 0; st < nfull; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) fetch((st + 1) * kLK);
    ld(buf, 0, 0);
#pragma unroll
    for (int kb = 0; kb < kLK; kb += 16) {
      const int s = (kb / 16) & 1;
      if (kb + 16 < kLK) ld(buf, s ^ 1, kb + 16);
      mma(s);
    }
    if (st + 1 < nst) put(buf ^ 1);
    __syncthreads();
  }
  // the partial last stage (K a multiple of 16): its remaining blocks
  for (int b = 0; b < tail; ++b) {
    ld(nfull & 1, 0, 16 * b);
    mma(0);
  }
  if (tail) __syncthreads();  // the epilogue tile reuses the stage buffers
  static_assert(kLN * kLTld <= 2 * kLM * kLLd, "tile fits the A stage buffers");
  float* tile = &sa[0][0];  // [kLN][kLTld] over both A stage buffers, free after the K loop
#pragma unroll
  for (int i = 0; i < kLTM; ++i)
#pragma unroll
    for (int j = 0; j < kLTN; ++j)
      *reinterpret_cast<f32x4*>(&tile[((wr * kLTN + j) * 16 + c) * kLTld + (wf * kLTM + i) * 16 + 4 * g]) = acc[i][j];
  __syncthreads();
  lgemm_epilogue<MODE>(a, l, mb, nb, tile, sb[0], red, in);
}

// ---- host plan ---------------------------------------------------------------------------------
struct Plan {
  MArgs a;
  int rt;
  size_t lds;
  int64_t ws_bytes;
  int64_t op_bytes, f32_off, f64_off;
  unsigned fb_grid, pack_grid, wgrad_grid;
};

int64_t roundup(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

int32_t make_plan(const smc_cvnn_layer* layers, int32_t n_layers, int32_t mode, int64_t batch, int64_t n_params,
                  Plan* out) {
  if (mode != SMC_CVNN_MFMA_F32 && mode != SMC_CVNN_MFMA_BF16)
    return fail(SMC_ERR_INVALID_ARGUMENT, "cvnn mfma: mode must be SMC_CVNN_MFMA_F32 or SMC_CVNN_MFMA_BF16");
  if (!layers || n_layers <= 0 || n_layers > kMaxL || batch <= 0)
    return fail(SMC_ERR_INVALID_SHAPE, "cvnn mfma: 1..SMC_CVNN_MAX_LAYERS layers and a positive batch");
  const bool bf16 = mode == SMC_CVNN_MFMA_BF16;
  const int KB = bf16 ? OpBf16::KB : OpF32::KB;
  const size_t es = bf16 ? 2 : 4;
  Plan p{};
  MArgs& a = p.a;
  a.n_layers = n_layers;
  a.batch = batch;
  a.n_params = n_params;
  int wmax = 0;
  for (int l = 0; l < n_layers; ++l) {
    const smc_cvnn_layer& s = layers[l];
    if (s.in_features <= 0 || s.out_features <= 0 || (l > 0 && s.in_features != layers[l - 1].out_features))
      return fail(SMC_ERR_INVALID_SHAPE, "cvnn mfma: inconsistent layer table");
    MLayer& m = a.layer[l];
    m.ni = s.in_features;
    m.no = s.out_features;
    m.act = s.activation;
    m.win = static_cast<int32_t>(roundup(2 * m.ni, KB));
    m.wout = static_cast<int32_t>(roundup(2 * m.no, KB));
    m.kx = static_cast<int32_t>(roundup(2 * m.ni + 1, 16));
    m.w_re = s.w_re;
    m.w_im = s.w_im;
    m.b_re = s.b_re;
    m.b_im = s.b_im;
    m.act_bias = s.act_bias;
    wmax = m.win > wmax ? m.win : wmax;
  }
  const int wlast = a.layer[n_layers - 1].wout;
  // wide layers (2 H >= 256, f32): the layered GEMM launches instead of fb_kernel
  a.layered = !bf16 && wmax >= 256 ? 1 : 0;
  a.lpb = 1;
  // LDS: split-K scratch [waves][RT][64] f32x4, two activation / gradient buffers [R][zs] and the last
  // layer's output gradient [R][gs]; row strides are odd multiples of 16 bytes (conflict-free
  // 16-byte fragment reads)
  a.zs = static_cast<int32_t>(wmax + 16 / es);
  a.gs = static_cast<int32_t>(wlast + 16 / es);
  size_t pre_floats = 0;  // pre-activations of the hidden layers with an activation, per row
  for (int l = 0; l + 1 < n_layers; ++l)
    if (a.layer[l].act != SMC_ACT_NONE) pre_floats += 2 * static_cast<size_t>(a.layer[l].no);
  size_t per16 = 16 * ((2 * static_cast<size_t>(a.zs) + a.gs) * es + pre_floats * 4) + kFbWaves * 64 * 16;
  a.pre_global = 0;
  if (per16 > kLdsCap) {  // pre-activations to the workspace instead
    a.pre_global = 1;
    per16 -= 16 * pre_floats * 4;
  }
  if (a.layered) {
    a.pre_global = 1;
    p.rt = 1;
    a.rows = kLN;  // batch rows per block (modReLU and loss partials)
    p.lds = 0;
    a.lpb = (wlast + kLM - 1) / kLM;
  } else {
    if (per16 > kLdsCap) return fail(SMC_ERR_INVALID_SHAPE, "cvnn mfma: layer widths exceed the LDS budget");
    p.rt = 2 * per16 <= kLdsPair && batch >= 4096 ? 2 : 1;
    a.rows = 16 * p.rt;
    p.lds = per16 * p.rt;
  }
  // batch segments of the weight gradients: powers of two, >= kSegmentRows rows each, until the
  // (feature tile, column-tile group, segment) items fill the chip
  int64_t blocks = 0;  // weight-gradient output blocks (64 x 64) of one segment
  for (int l = 0; l < n_layers; ++l)
    blocks += ((a.layer[l].wout + kWgBlock - 1) / kWgBlock) * static_cast<int64_t>((a.layer[l].kx + kWgBlock - 1) / kWgBlock);
  int segs = 1;
  while (segs < kMaxSegments && batch / (2 * segs) >= kSegmentRows && blocks * 2 * segs <= kWgradBlocks) segs *= 2;
  a.segs = segs;
  const int64_t unit = roundup(a.rows, kWgStage);  // powers of two: the rows and a K stage divide it
  a.bp = roundup(batch, unit * segs);
  a.nwg = static_cast<int32_t>(a.bp / a.rows);
  // workspace: Op region (packed weights, Z^T, dU^T), f32 region (pre-activations, modReLU partials), f64 (loss)
  int64_t op = 0;
  a.pack_elems = 0;
  for (int l = 0; l < n_layers; ++l) {
    MLayer& m = a.layer[l];
    const int64_t kc = a.layered ? m.kx : m.win;  // layered: Wc with the bias column
    m.wc = op;
    op += static_cast<int64_t>(m.wout) * kc;
    m.wct = op;
    op += static_cast<int64_t>(m.wout) * m.win;
    a.pack_elems += static_cast<int64_t>(m.wout) * (kc + m.win);
  }
  if (a.layered) a.pack_elems += 2 * a.bp * a.layer[0].kx;  // Z_0 and Z_0^T
  for (int l = 0; l < n_layers; ++l) {
    MLayer& m = a.layer[l];
    op = roundup(op, 64);
    m.zt = op;
    op += static_cast<int64_t>(m.kx) * a.bp;
    op = roundup(op, 64);
    m.gt = op;
    op += static_cast<int64_t>(m.wout) * a.bp;
    m.zr = m.dr = -1;
    if (a.layered) {
      op = roundup(op, 64);
      m.zr = op;
      op += static_cast<int64_t>(m.kx) * a.bp;
      op = roundup(op, 64);
      m.dr = op;
      op += static_cast<int64_t>(m.wout) * a.bp;
    }
  }
  p.op_bytes = roundup(op * static_cast<int64_t>(es), 256);
  int64_t f = 0, pre_off = 0;
  for (int l = 0; l < n_layers; ++l) {
    MLayer& m = a.layer[l];
    m.pre = -1;
    m.cpart = -1;
    if (l + 1 < n_layers && m.act != SMC_ACT_NONE) {
      if (a.pre_global) {
        m.pre = f;
        f = roundup(f + a.bp * 2 * m.no, 64);
      } else {
        m.pre = pre_off;
        pre_off += static_cast<int64_t>(a.rows) * 2 * m.no;
      }
    }
    if (m.act == SMC_ACT_MODRELU) {
      m.cpart = f;
      f = roundup(f + static_cast<int64_t>(a.nwg) * m.no, 64);
    }
    m.items = ((m.wout + kWgBlock - 1) / kWgBlock) * static_cast<int64_t>((m.kx + kWgBlock - 1) / kWgBlock) * a.segs;
  }
  p.f32_off = p.op_bytes;
  p.f64_off = roundup(p.f32_off + f * 4, 256);
  p.ws_bytes = p.f64_off + static_cast<int64_t>(a.nwg) * a.lpb * 8;
  int64_t items = (a.segs + kWaves - 1) / kWaves;  // bookkeeping workgroups (one segment per wave)
  for (int l = 0; l < n_layers; ++l) items += a.layer[l].items;
  p.fb_grid = static_cast<unsigned>(a.nwg);
  p.wgrad_grid = static_cast<unsigned>(items);
  const int64_t pg = (a.pack_elems + kThreads - 1) / kThreads;
  p.pack_grid = static_cast<unsigned>(pg < 2048 ? pg : 2048);
  *out = p;
  return SMC_OK;
}

template <class Op, int RT>
int32_t launch_fb(const Plan& p, hipStream_t s) {
  auto kernel = fb_kernel<Op, RT>;
  if (p.lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          static_cast<int>(p.lds)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "cvnn fb_kernel: cannot raise the dynamic LDS limit");
  }
  hipLaunchKernelGGL(kernel, dim3(p.fb_grid), dim3(kFbThreads), p.lds, s, p.a);
  return SMC_OK;
}

int32_t launch_layered(const Plan& p, hipStream_t s) {
  const MArgs& a = p.a;
  // (row-major wgrad: no Z_0^T region)
  hipLaunchKernelGGL(lpack_kernel, dim3(256, 2 * a.n_layers + (kWgradRowMajor ? 1 : 2)), dim3(kThreads), 0, s, a);
  if (int32_t rc = check_launch("cvnn lpack_kernel")) return rc;
  const unsigned by = static_cast<unsigned>(a.bp / kLN);
  const int L = a.n_layers;
  MArgs g = a;  // lgemm_mb: the launch's feature blocks (1-D grid of lgemm_mb x (by rounded to 8) workgroups)
  const unsigned byx = (by + 7) / 8 * 8;
  for (int l = 0; l < L; ++l) {
    g.lgemm_mb = (a.layer[l].wout + kLM - 1) / kLM;
    const dim3 grid(static_cast<unsigned>(g.lgemm_mb) * byx);
    if (l + 1 < L) hipLaunchKernelGGL(lgemm_kernel<kLFwd>, grid, dim3(kLThreads), 0, s, g, l);
    else hipLaunchKernelGGL(lgemm_kernel<kLLast>, grid, dim3(kLThreads), 0, s, g, l);
    if (int32_t rc = check_launch("cvnn lgemm_kernel")) return rc;
  }
  for (int l = L - 1; l >= 1; --l) {
    g.lgemm_mb = (a.layer[l].win + kLM - 1) / kLM;
    const dim3 grid(static_cast<unsigned>(g.lgemm_mb) * byx);
    hipLaunchKernelGGL(lgemm_kernel<kLBwd>, grid, dim3(kLThreads), 0, s, g, l);
    if (int32_t rc = check_launch("cvnn lgemm_kernel")) return rc;
  }
  // weight gradients in wgrad_kernel's 64 x 64 blocks over batch segments (they measured faster here than
  // this file's GEMM tile: 70 vs 74-81 us at C2/H=256), from the row-major Z_l / dU_l (wgrad_rm_kernel,
  // round 4) or, without kWgradRowMajor, from ^T copies as after fb_kernel
  if (kWgradRowMajor)
    hipLaunchKernelGGL(wgrad_rm_kernel<kWgradKsF32>, dim3(p.wgrad_grid), dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL(wgrad_kernel<OpF32>, dim3(p.wgrad_grid), dim3(kThreads), 0, s, a);
  return check_launch("cvnn wgrad_kernel");
}

template <class Op>
int32_t launch_all(const Plan& p, hipStream_t s, bool packed) {
  if (p.a.layered) return launch_layered(p, s);
  if (!packed) {  // (packed: the last Adam update wrote the operand copies, smc_cvnn_pack)
    hipLaunchKernelGGL(pack_kernel<Op>, dim3(p.pack_grid), dim3(kThreads), 0, s, p.a);
    if (int32_t rc = check_launch("cvnn pack_kernel")) return rc;
  }
  if (int32_t rc = p.rt == 2 ? launch_fb<Op, 2>(p, s) : launch_fb<Op, 1>(p, s)) return rc;
  if (int32_t rc = check_launch("cvnn fb_kernel")) return rc;
  hipLaunchKernelGGL(wgrad_kernel<Op>, dim3(p.wgrad_grid), dim3(kThreads), 0, s, p.a);
  return check_launch("cvnn wgrad_kernel");
}

}  // namespace
}  // namespace smc

using namespace smc;

#pragma GCC visibility push(default)
extern "C" {

int32_t smc_cvnn_mfma_plan(const smc_cvnn_layer* layers, int32_t n_layers, int32_t mode, int64_t batch,
                           int64_t* partial_blocks, int64_t* workspace_bytes) {
  if (!partial_blocks || !workspace_bytes) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_cvnn_mfma_plan: null output");
  Plan p;
  const int32_t rc = make_plan(layers, n_layers, mode, batch, 0, &p);
  if (rc != SMC_OK) return rc;
  *partial_blocks = p.a.segs;
  *workspace_bytes = p.ws_bytes;
  return SMC_OK;
}

int32_t smc_cvnn_mfma_forward_backward(const smc_cvnn_layer* layers, int32_t n_layers, int32_t mode,
                                       const float* params, int64_t n_params, const float* input_re,
                                       const float* input_im, const void* targets, int64_t batch, float* partials,
                                       int64_t partial_blocks, void* workspace, int64_t workspace_bytes,
                                       void* stream) {
  if (!params || !input_re || !targets || !partials || !workspace || n_params <= 0)
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_cvnn_mfma_forward_backward: bad argument");
  for (int l = 0; layers && l < n_layers && l < kMaxL; ++l) {
    const smc_cvnn_layer& s = layers[l];
    const int64_t w = static_cast<int64_t>(s.in_features) * s.out_features;
    bool ok = s.activation >= SMC_ACT_NONE && s.activation <= SMC_ACT_ZRELU && s.w_re >= 0 && s.w_im >= 0 &&
              s.w_re + w <= n_params && s.w_im + w <= n_params;
    for (int64_t o : {s.b_re, s.b_im}) ok = ok && (o < 0 || o + s.out_features <= n_params);
    if (s.activation == SMC_ACT_MODRELU) ok = ok && s.act_bias >= 0 && s.act_bias + s.out_features <= n_params;
    if (!ok) return fail(SMC_ERR_INVALID_SHAPE, "smc_cvnn_mfma_forward_backward: inconsistent layer table");
  }
  const bool packed = (mode & SMC_CVNN_MFMA_PACKED) != 0;
  mode &= ~SMC_CVNN_MFMA_PACKED;
  Plan p;
  const int32_t rc = make_plan(layers, n_layers, mode, batch, n_params, &p);
  if (rc != SMC_OK) return rc;
  if (partial_blocks != p.a.segs) return fail(SMC_ERR_INVALID_SHAPE, "smc_cvnn_mfma_forward_backward: partial_blocks != plan");
  if (workspace_bytes < p.ws_bytes) return fail(SMC_ERR_INVALID_SHAPE, "smc_cvnn_mfma_forward_backward: workspace too small");
  MArgs& a = p.a;
  a.params = params;
  a.in_re = input_re;
  a.in_im = input_im;
  a.targets = static_cast<const float*>(targets);
  a.opws = workspace;
  a.fws = reinterpret_cast<float*>(static_cast<char*>(workspace) + p.f32_off);
  a.lossp = reinterpret_cast<double*>(static_cast<char*>(workspace) + p.f64_off);
  a.partials = partials;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  return mode == SMC_CVNN_MFMA_BF16 ? launch_all<OpBf16>(p, s, packed) : launch_all<OpF32>(p, s, packed);
}

int32_t smc_cvnn_mfma_pack_plan(const smc_cvnn_layer* layers, int32_t n_layers, int32_t mode, int64_t batch,
                                void* workspace, smc_cvnn_pack* out) {
  if (!out || !workspace) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_cvnn_mfma_pack_plan: null argument");
  Plan p;
  const int32_t rc = make_plan(layers, n_layers, mode, batch, 0, &p);
  if (rc != SMC_OK) return rc;
  *out = smc_cvnn_pack{};
  out->ws = workspace;
  out->bf16 = mode == SMC_CVNN_MFMA_BF16 ? 1 : 0;
  if (p.a.layered) return SMC_OK;  // the layered GEMM path packs Wc with its bias column itself
  out->n_layers = n_layers;
  for (int l = 0; l < n_layers; ++l) {
    const MLayer& m = p.a.layer[l];
    out->layer[l] = smc_cvnn_pack_layer{layers[l].w_re, layers[l].w_im, m.ni, m.no, m.win, m.wout, m.wc, m.wct};
  }
  return SMC_OK;
}

}  // extern "C"
#pragma GCC visibility pop
