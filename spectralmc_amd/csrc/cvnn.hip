// Complex-valued MLP training step for gfx950: forward, spectral MSE, backward and Adam in
// three launches (torch-ROCm issues ~200 small kernels for the same step).
//
// Reference behaviour restated (Tuee22/SpectralMC, src/spectralmc/):
//   cvnn.py:65-143   ComplexLinear  u = A x - B y + b_re,  v = B x + A y + b_im
//   cvnn.py:149-162  zReLU          keep z where Re z >= 0 and Im z >= 0
//   cvnn.py:168-210  modReLU        m = sqrt(u^2 + v^2 + 1e-9),  z * relu(m + c) / m
//   gbm_trainer.py:819-835  loss = mse(pred_re, Re y) + mse(pred_im, Im y); backward;
//                    Adam.step (torch defaults); grad_norm = ||g||_2 after the step
//
// Design:
//   * forward_backward_kernel: a workgroup takes blocks of R rows, keeps every layer's
//     pre-activation and output for those rows in LDS, back-propagates through them and adds
//     the rows' weight gradients into its own slot of a partial buffer [G][n_params + 1]
//     (the last entry is the loss).  Fixed row-block assignment and fixed loop orders make
//     the result bit-reproducible; no float atomics.
//   * reduce_kernel: one thread per parameter sums the G partials in order (f64) -> flat
//     gradient buffer [n_params + 1]; with SMC Adam arguments it also applies the Adam update
//     (fused, single process) and per-block partial sums of g^2.
//   * adam_kernel: the same update from an already reduced (all-reduced) gradient buffer.
//   * the last workgroup of either (an arrival counter) takes the grad norm from the block partials (fixed
//     order), the loss and step += 1; reduce grids above kFuseFinalizeMaxBlocks workgroups (wide networks)
//     leave that to finalize_kernel, a one-workgroup launch.
// Weights stay in HBM/L2 (tens of KB for the benchmark network); parameters, gradients and
// Adam moments are single flat buffers whose layout is the model's parameter order.

#include <cmath>

#include "smc_device.h"
#include "smc_internal.h"

namespace smc {
namespace {

constexpr int kNetThreads = 256;
constexpr int kMaxLayers = SMC_CVNN_MAX_LAYERS;
constexpr int kMaxBlocks = 256;       // partial slots (workgroups) of forward_backward_kernel
constexpr size_t kNetLdsBudget = 96 * 1024;  // leaves room for two contract_kernel workgroups per CU

struct NetArgs {
  int32_t n_layers;
  smc_cvnn_layer layer[kMaxLayers];
  int32_t rows;             // R rows per row block
  int64_t batch;
  int64_t n_params;
  int32_t out_features;     // N of the last layer
  const void* params;
  const void* input_re;     // [B][n_in0]
  const void* input_im;     // [B][n_in0] or NULL (zeros)
  const void* targets;      // [B][N] complex (interleaved re, im)
  void* partials;           // [G][n_params + 1]
};

// LDS layout per row block (element offsets, multiplied by rows):
//   in0_re, in0_im          n_in0 each
//   per layer l: u, v       n_out each   (pre-activation)
//                ar, ai     n_out each   (activation output; only if activation != none)
//   g0_re, g0_im, g1_re, g1_im   max width each (gradient ping-pong)
struct LdsPlan {
  int64_t in_re, in_im;
  int64_t u[kMaxLayers], v[kMaxLayers], ar[kMaxLayers], ai[kMaxLayers];
  int64_t g[4];
  int64_t scratch;          // input-gradient partials: 2 * max(kNetThreads, widest input)
  int64_t per_row;
};

__host__ __device__ inline void plan_lds_into(const smc_cvnn_layer* layer, int n_layers, LdsPlan* out) {
  LdsPlan& p = *out;
  int64_t off = 0;
  const int n0 = layer[0].in_features;
  p.in_re = off;
  off += n0;
  p.in_im = off;
  off += n0;
  int wmax = n0;
  for (int l = 0; l < n_layers; ++l) {
    const int n = layer[l].out_features;
    wmax = n > wmax ? n : wmax;
    p.u[l] = off;
    off += n;
    p.v[l] = off;
    off += n;
    if (layer[l].activation != SMC_ACT_NONE) {
      p.ar[l] = off;
      off += n;
      p.ai[l] = off;
      off += n;
    } else {
      p.ar[l] = p.u[l];
      p.ai[l] = p.v[l];
    }
  }
  for (int k = 0; k < 4; ++k) {
    p.g[k] = off;
    off += wmax;
  }
  p.scratch = off;
  off += 2 * (wmax > kNetThreads ? wmax : kNetThreads);
  p.per_row = off;
}

inline LdsPlan plan_lds(const smc_cvnn_layer* layer, int n_layers) {
  LdsPlan p{};
  plan_lds_into(layer, n_layers, &p);
  return p;
}

template <typename Real>
__device__ __forceinline__ Real block_sum(Real x, double* red_raw) {
  Real* red = reinterpret_cast<Real*>(red_raw);
  // fixed-order block reduction: wave butterfly, then waves 0..3 in order
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = x;
  __syncthreads();
  Real t = 0;
  for (int w = 0; w < kNetThreads / 64; ++w) t += red[w];
  return t;
}

// Forward + backward of R-row blocks.  Register blocking over the R rows: each weight is
// loaded once per row block (forward: thread per output feature; input gradients: thread per
// (input feature, j-group) with a fixed-order LDS reduction over the groups).
template <typename Real, int R>
__global__ __launch_bounds__(kNetThreads) void forward_backward_kernel(NetArgs a) {
  extern __shared__ double net_lds_raw[];
  Real* lds = reinterpret_cast<Real*>(net_lds_raw);
  const int tid = threadIdx.x;
  const int L = a.n_layers;
  // layer table and LDS plan in LDS: indexed by the runtime layer number, they would otherwise
  // be copied to scratch memory
  __shared__ smc_cvnn_layer layer[kMaxLayers];
  __shared__ LdsPlan pl;
  __shared__ double red[kNetThreads / 64];
  if (tid == 0) {
#pragma unroll
    for (int i = 0; i < kMaxLayers; ++i) layer[i] = a.layer[i];  // compile-time indices: no scratch copy
  }
  __syncthreads();
  if (tid == 0) plan_lds_into(layer, L, &pl);
  __syncthreads();
  const Real* P = static_cast<const Real*>(a.params);
  Real* part = static_cast<Real*>(a.partials) + static_cast<int64_t>(blockIdx.x) * (a.n_params + 1);
  const Real* in_re = static_cast<const Real*>(a.input_re);
  const Real* in_im = static_cast<const Real*>(a.input_im);
  const Real* tgt = static_cast<const Real*>(a.targets);
  const int n0 = layer[0].in_features;
  const int N = a.out_features;
  const Real scale = Real(2) / static_cast<Real>(static_cast<double>(a.batch) * N);  // d mean / d x
  double loss_acc = 0.0;
  const int64_t n_blocks = (a.batch + R - 1) / R;
  bool first = true;

  for (int64_t rb = blockIdx.x; rb < n_blocks; rb += gridDim.x, first = false) {
    const int64_t r0 = rb * R;
    const int rows = static_cast<int>(a.batch - r0 < R ? a.batch - r0 : R);
    // ---- load inputs (rows >= `rows` are zero-filled so unused lanes of the blocking stay finite)
    for (int i = tid; i < R * n0; i += kNetThreads) {
      const bool ok = i < rows * n0;
      lds[pl.in_re * R + i] = ok ? in_re[r0 * n0 + i] : Real(0);
      lds[pl.in_im * R + i] = ok && in_im ? in_im[r0 * n0 + i] : Real(0);
    }
    __syncthreads();
    // ---- forward
    for (int l = 0; l < L; ++l) {
      const smc_cvnn_layer& ly = layer[l];
      const int ni = ly.in_features, no = ly.out_features;
      const Real* x = lds + (l == 0 ? pl.in_re : pl.ar[l - 1]) * R;
      const Real* y = lds + (l == 0 ? pl.in_im : pl.ai[l - 1]) * R;
      Real* u = lds + pl.u[l] * R;
      Real* v = lds + pl.v[l] * R;
      for (int j = tid; j < no; j += kNetThreads) {
        Real au[R], av[R];
        const Real br = ly.b_re >= 0 ? P[ly.b_re + j] : Real(0);
        const Real bi = ly.b_im >= 0 ? P[ly.b_im + j] : Real(0);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          au[r] = br;
          av[r] = bi;
        }
        const Real* Aj = P + ly.w_re + static_cast<int64_t>(j) * ni;
        const Real* Bj = P + ly.w_im + static_cast<int64_t>(j) * ni;
        for (int k = 0; k < ni; ++k) {
          const Real wa = Aj[k], wb = Bj[k];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const Real xr = x[r * ni + k], yr = y[r * ni + k];
            au[r] += wa * xr - wb * yr;
            av[r] += wb * xr + wa * yr;
          }
        }
        const Real c = ly.activation == SMC_ACT_MODRELU ? P[ly.act_bias + j] : Real(0);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int idx = r * no + j;
          const Real su = au[r], sv = av[r];
          u[idx] = su;
          v[idx] = sv;
          if (ly.activation == SMC_ACT_MODRELU) {
            const Real m = sqrt(su * su + sv * sv + Real(1e-9));
            const Real t = m + c;
            const Real g = (t > Real(0) ? t : Real(0)) / m;
            lds[pl.ar[l] * R + idx] = g * su;
            lds[pl.ai[l] * R + idx] = g * sv;
          } else if (ly.activation == SMC_ACT_ZRELU) {
            const bool keep = su >= Real(0) && sv >= Real(0);
            lds[pl.ar[l] * R + idx] = keep ? su : Real(0);
            lds[pl.ai[l] * R + idx] = keep ? sv : Real(0);
          }
        }
      }
      __syncthreads();
    }
    // ---- loss and d loss / d prediction (rows >= `rows` get zero gradient)
    {
      const Real* pr = lds + pl.ar[L - 1] * R;
      const Real* pi = lds + pl.ai[L - 1] * R;
      Real* gr = lds + pl.g[0] * R;
      Real* gi = lds + pl.g[1] * R;
      double part_loss = 0.0;
      for (int idx = tid; idx < R * N; idx += kNetThreads) {
        const int r = idx / N, j = idx - r * N;
        if (r < rows) {
          const int64_t t = ((r0 + r) * N + j) * 2;
          const Real dr = pr[idx] - tgt[t];
          const Real di = pi[idx] - tgt[t + 1];
          part_loss += static_cast<double>(dr * dr) + static_cast<double>(di * di);
          gr[idx] = scale * dr;
          gi[idx] = scale * di;
        } else {
          gr[idx] = Real(0);
          gi[idx] = Real(0);
        }
      }
      loss_acc += block_sum<double>(part_loss, red);
    }
    __syncthreads();
    // ---- backward
    int cur = 0;  // g[cur], g[cur+1]: gradient w.r.t. the current layer's output (re, im)
    for (int l = L - 1; l >= 0; --l) {
      const smc_cvnn_layer& ly = layer[l];
      const int ni = ly.in_features, no = ly.out_features;
      Real* go_r = lds + pl.g[cur] * R;
      Real* go_i = lds + pl.g[cur + 1] * R;
      const Real* u = lds + pl.u[l] * R;
      const Real* v = lds + pl.v[l] * R;
      if (ly.activation == SMC_ACT_MODRELU) {
        // d/dc first (needs the output gradient), then the output gradient -> (gu, gv) in place
        for (int j = tid; j < no; j += kNetThreads) {
          const Real c = P[ly.act_bias + j];
          Real s = 0;
          for (int r = 0; r < rows; ++r) {
            const int idx = r * no + j;
            const Real m = sqrt(u[idx] * u[idx] + v[idx] * v[idx] + Real(1e-9));
            if (m + c > Real(0)) s += (go_r[idx] * u[idx] + go_i[idx] * v[idx]) / m;
          }
          Real* dst = part + ly.act_bias + j;
          *dst = first ? s : *dst + s;
        }
        __syncthreads();
        for (int idx = tid; idx < R * no; idx += kNetThreads) {
          const int j = idx % no;
          const Real c = P[ly.act_bias + j];
          const Real uu = u[idx], vv = v[idx];
          const Real m = sqrt(uu * uu + vv * vv + Real(1e-9));
          if (m + c > Real(0)) {
            const Real g = (m + c) / m;
            const Real k = -(go_r[idx] * uu + go_i[idx] * vv) * c / (m * m * m);
            go_r[idx] = go_r[idx] * g + k * uu;
            go_i[idx] = go_i[idx] * g + k * vv;
          } else {
            go_r[idx] = Real(0);
            go_i[idx] = Real(0);
          }
        }
        __syncthreads();
      } else if (ly.activation == SMC_ACT_ZRELU) {
        for (int idx = tid; idx < R * no; idx += kNetThreads) {
          if (!(u[idx] >= Real(0) && v[idx] >= Real(0))) {
            go_r[idx] = Real(0);
            go_i[idx] = Real(0);
          }
        }
        __syncthreads();
      }
      const Real* x = lds + (l == 0 ? pl.in_re : pl.ar[l - 1]) * R;
      const Real* y = lds + (l == 0 ? pl.in_im : pl.ai[l - 1]) * R;
      // weight gradients: dA = gu x^T + gv y^T,  dB = gv x^T - gu y^T  (summed over the rows)
      for (int idx = tid; idx < no * ni; idx += kNetThreads) {
        const int j = idx / ni, k = idx - j * ni;
        Real da = 0, db = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const Real gu = go_r[r * no + j], gv = go_i[r * no + j];
          const Real xk = x[r * ni + k], yk = y[r * ni + k];
          da += gu * xk + gv * yk;
          db += gv * xk - gu * yk;
        }
        Real* pa = part + ly.w_re + idx;
        Real* pb = part + ly.w_im + idx;
        *pa = first ? da : *pa + da;
        *pb = first ? db : *pb + db;
      }
      for (int j = tid; j < no; j += kNetThreads) {
        Real sr = 0, si = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          sr += go_r[r * no + j];
          si += go_i[r * no + j];
        }
        if (ly.b_re >= 0) part[ly.b_re + j] = first ? sr : part[ly.b_re + j] + sr;
        if (ly.b_im >= 0) part[ly.b_im + j] = first ? si : part[ly.b_im + j] + si;
      }
      if (l > 0) {
        // input gradients gx = A^T gu + B^T gv, gy = A^T gv - B^T gu: thread (g, k) sums the
        // j = g, g+G, ... terms for all R rows; the G partials are added in order after a barrier
        Real* gx = lds + pl.g[2 - cur] * R;
        Real* gy = lds + pl.g[3 - cur] * R;
        Real* scr = lds + pl.scratch * R;
        const int G = ni >= kNetThreads ? 1 : kNetThreads / ni;
        const Real* A = P + ly.w_re;
        const Real* Bw = P + ly.w_im;
        for (int t = tid; t < G * ni; t += kNetThreads) {
          const int g = t / ni, k = t - g * ni;
          Real sx[R], sy[R];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            sx[r] = Real(0);
            sy[r] = Real(0);
          }
          for (int j = g; j < no; j += G) {
            const Real wa = A[static_cast<int64_t>(j) * ni + k], wb = Bw[static_cast<int64_t>(j) * ni + k];
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const Real gu = go_r[r * no + j], gv = go_i[r * no + j];
              sx[r] += wa * gu + wb * gv;
              sy[r] += wa * gv - wb * gu;
            }
          }
#pragma unroll
          for (int r = 0; r < R; ++r) {
            scr[(static_cast<int64_t>(r) * G + g) * ni + k] = sx[r];
            scr[(static_cast<int64_t>(R + r) * G + g) * ni + k] = sy[r];
          }
        }
        __syncthreads();
        for (int idx = tid; idx < R * ni; idx += kNetThreads) {
          const int r = idx / ni, k = idx - r * ni;
          Real sx = 0, sy = 0;
          for (int g = 0; g < G; ++g) {
            sx += scr[(static_cast<int64_t>(r) * G + g) * ni + k];
            sy += scr[(static_cast<int64_t>(R + r) * G + g) * ni + k];
          }
          gx[idx] = sx;
          gy[idx] = sy;
        }
        cur = 2 - cur;
      }
      __syncthreads();
    }
  }
  if (tid == 0) part[a.n_params] = static_cast<Real>(loss_acc / (static_cast<double>(a.batch) * N));
}

struct AdamArgs {
  void* params;
  void* exp_avg;
  void* exp_avg_sq;
  float* step;  // torch's capturable step counter before this update (the last workgroup increments it)
  double lr, beta1, beta2, eps, weight_decay;
  double* norm_partials;  // [gridDim] sums of g^2, then (at norm_slots - 1) the arrival counter
  int64_t norm_slots;     // smc_adam_norm_partials(n_params)
  void* grad_norm;        // scalar out
  void* loss;             // scalar out: grads[n_params]
  int32_t fuse_final;     // the last workgroup finalizes (else finalize_kernel, a launch of its own)
  smc_cvnn_pack pack;     // packed MFMA operand copies the update also writes (n_layers = 0: none)
};

// Reduce grids up to this many workgroups finalize in their last workgroup; larger ones in finalize_kernel:
// every workgroup's drained sc1 hand-off and one counter atomic cost more than the launch they save (round 5:
// the H = 256 network's 4,176-workgroup reduce alone 0.224 -> 0.266 ms fused; the narrow networks' <= 306
// workgroups: e2e 0.108 -> 0.098 ms/step, lock-step 0.305 -> 0.295, profiles/r05/bench_finalize_sc1_vs_r4.txt)
constexpr int64_t kFuseFinalizeMaxBlocks = 1024;

// The MFMA operand copies of parameter p (smc_cvnn_pack, spectralmc_hip.h): cvnn_mfma.hip pack_kernel's
// layout, element for element -- w = a + i b of layer l at (j, k) is Wc[2j][2k] = Wc[2j+1][2k+1] = a,
// Wc[2j][2k+1] = -b, Wc[2j+1][2k] = b and the same entries of Wc^T; biases are not packed.
__device__ __forceinline__ void pack_weight(const smc_cvnn_pack& pk, int64_t p, float v) {
  for (int l = 0; l < pk.n_layers; ++l) {
    const smc_cvnn_pack_layer& L = pk.layer[l];
    const int64_t w = static_cast<int64_t>(L.ni) * L.no;
    const bool re = p >= L.w_re && p < L.w_re + w, im = p >= L.w_im && p < L.w_im + w;
    if (!re && !im) continue;
    const int64_t r = p - (re ? L.w_re : L.w_im);
    const int f = 2 * static_cast<int>(r / L.ni), k = 2 * static_cast<int>(r % L.ni);
    // (row f + df, column k + dk) of Wc: re at (0, 0) and (1, 1); im at (0, 1) negated and (1, 0)
    const int f0 = f, k0 = re ? k : k + 1, f1 = f + 1, k1 = re ? k + 1 : k;
    const float v0 = re ? v : -v;
    const int64_t c0 = L.wc + static_cast<int64_t>(f0) * L.win + k0, c1 = L.wc + static_cast<int64_t>(f1) * L.win + k1;
    const int64_t t0 = L.wct + static_cast<int64_t>(k0) * L.wout + f0, t1 = L.wct + static_cast<int64_t>(k1) * L.wout + f1;
    if (pk.bf16) {
      uint16_t* ws = static_cast<uint16_t*>(pk.ws);
      ws[c0] = ws[t0] = bf16_bits(v0);
      ws[c1] = ws[t1] = bf16_bits(v);
    } else {
      float* ws = static_cast<float*>(pk.ws);
      ws[c0] = ws[t0] = v0;
      ws[c1] = ws[t1] = v;
    }
    return;
  }
}

template <typename Real>
__device__ __forceinline__ void adam_update(const AdamArgs& ad, int64_t p, Real g) {
  Real* prm = static_cast<Real*>(ad.params);
  Real* m = static_cast<Real*>(ad.exp_avg);
  Real* v = static_cast<Real*>(ad.exp_avg_sq);
  const Real t = static_cast<Real>(*ad.step) + Real(1);
  const Real b1 = static_cast<Real>(ad.beta1), b2 = static_cast<Real>(ad.beta2);
  if (ad.weight_decay != 0.0) g += static_cast<Real>(ad.weight_decay) * prm[p];
  const Real mm = m[p] + (Real(1) - b1) * (g - m[p]);
  const Real vv = v[p] * b2 + (Real(1) - b2) * g * g;
  m[p] = mm;
  v[p] = vv;
  const Real bc1 = Real(1) - pow(b1, t);
  const Real bc2 = Real(1) - pow(b2, t);
  const Real step_size = static_cast<Real>(ad.lr) / bc1;
  const Real denom = sqrt(vv) / sqrt(bc2) + static_cast<Real>(ad.eps);
  const Real np = prm[p] - step_size * (mm / denom);
  prm[p] = np;
  if constexpr (sizeof(Real) == 4) {
    if (ad.pack.n_layers > 0) pack_weight(ad.pack, p, np);
  }
}

// One block = 64 consecutive gradient entries x 4 slices of the G partials (a wave per slice,
// so every load instruction reads 64 consecutive entries); slices are added in order.
constexpr int kReduceCols = 64;
constexpr int kReduceSlices = kNetThreads / kReduceCols;

// The update's tail, fused (round 5: it was a separate one-workgroup finalize_kernel launch): every workgroup
// publishes its g^2 partial; the last one to arrive on the counter (the final slot of norm_partials, zero between
// launches) adds the partials in index order (finalize_kernel's order: thread stride, then block_sum), writes the
// grad norm and the loss, increments Adam's step and resets the counter.  Every workgroup read the step before
// it arrived.  Hand-off without fences: the partial (and the loss slot, reduce_kernel) are write-through (sc1)
// stores drained before the arrival and read with sc1 loads (MI355X_MICROARCH.md, inter-workgroup visibility).
// An agent-scope release fence per thread would write back the XCD's whole L2 -- beside the path kernel, all of
// its dirty path lines: the first fused form (__threadfence per thread) made the H = 256 network 0.22 -> 0.53 ms.
template <typename Real>
__device__ __forceinline__ void adam_finalize_last(const AdamArgs& ad, int64_t n_partials, const Real* grads,
                                                   int64_t n_params, double* red, double partial) {
  __shared__ int last;
  if (threadIdx.x == 0) put_sc1(ad.norm_partials + blockIdx.x, partial);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores (the partial, the loss slot) done
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t* cnt = reinterpret_cast<uint32_t*>(ad.norm_partials + (ad.norm_slots - 1));
    last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  double sum = 0.0;
  for (int64_t i = threadIdx.x; i < n_partials; i += kNetThreads) sum += get_sc1(ad.norm_partials + i);
  const double t = block_sum<double>(sum, red);
  if (threadIdx.x == 0) {
    *static_cast<Real*>(ad.grad_norm) = static_cast<Real>(sqrt(t));
    *static_cast<Real*>(ad.loss) = get_sc1(grads + n_params);
    *ad.step = *ad.step + 1.0f;
    __hip_atomic_store(reinterpret_cast<uint32_t*>(ad.norm_partials + (ad.norm_slots - 1)), 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <typename Real, bool ADAM>
__global__ __launch_bounds__(kNetThreads) void reduce_kernel(const Real* __restrict__ partials, int64_t blocks,
                                                             int64_t n_params, Real* __restrict__ grads,
                                                             AdamArgs ad) {
  __shared__ double red[kNetThreads / 64];
  __shared__ double slice_sum[kReduceSlices][kReduceCols];
  const int col = threadIdx.x % kReduceCols, slice = threadIdx.x / kReduceCols;
  const int64_t p = static_cast<int64_t>(blockIdx.x) * kReduceCols + col;
  const int64_t stride = n_params + 1;
  double s0 = 0.0, s1 = 0.0;
  if (p <= n_params) {
    int64_t g = slice;
    for (; g + kReduceSlices < blocks; g += 2 * kReduceSlices) {
      s0 += static_cast<double>(partials[g * stride + p]);
      s1 += static_cast<double>(partials[(g + kReduceSlices) * stride + p]);
    }
    for (; g < blocks; g += kReduceSlices) s0 += static_cast<double>(partials[g * stride + p]);
  }
  slice_sum[slice][col] = s0 + s1;
  __syncthreads();
  double sq = 0.0;
  if (slice == 0 && p <= n_params) {
    double s = 0.0;
    for (int k = 0; k < kReduceSlices; ++k) s += slice_sum[k][col];
    const Real gr = static_cast<Real>(s);
    if (ADAM && p == n_params) put_sc1(grads + p, gr);  // the loss slot: read by the last workgroup
    else grads[p] = gr;
    if (ADAM && p < n_params) {
      sq = static_cast<double>(gr) * static_cast<double>(gr);
      adam_update<Real>(ad, p, gr);
    }
  }
  if (ADAM) {
    const double t = block_sum<double>(sq, red);
    if (ad.fuse_final) adam_finalize_last<Real>(ad, gridDim.x, grads, n_params, red, t);
    else if (threadIdx.x == 0) ad.norm_partials[blockIdx.x] = t;
  }
}

template <typename Real>
__global__ __launch_bounds__(kNetThreads) void adam_kernel(const Real* __restrict__ grads, int64_t n_params,
                                                           AdamArgs ad) {
  __shared__ double red[kNetThreads / 64];
  const int64_t p = static_cast<int64_t>(blockIdx.x) * kNetThreads + threadIdx.x;
  double sq = 0.0;
  if (p < n_params) {
    const Real g = grads[p];
    sq = static_cast<double>(g) * static_cast<double>(g);
    adam_update<Real>(ad, p, g);
  }
  const double t = block_sum<double>(sq, red);
  if (ad.fuse_final) adam_finalize_last<Real>(ad, gridDim.x, grads, n_params, red, t);
  else if (threadIdx.x == 0) ad.norm_partials[blockIdx.x] = t;
}

// The finalize of large reduce grids (!AdamArgs.fuse_final): grad norm from the block partials (fixed order),
// loss, step += 1, one workgroup after the update launch.
template <typename Real>
__global__ __launch_bounds__(kNetThreads) void finalize_kernel(const double* __restrict__ norm_partials,
                                                               int64_t n_partials, const Real* __restrict__ grads,
                                                               int64_t n_params, float* step, Real* grad_norm,
                                                               Real* loss) {
  __shared__ double red[kNetThreads / 64];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n_partials; i += kNetThreads) s += norm_partials[i];
  const double t = block_sum<double>(s, red);
  if (threadIdx.x == 0) {
    *grad_norm = static_cast<Real>(sqrt(t));
    *loss = grads[n_params];
    *step = *step + 1.0f;
  }
}

template <typename Real>
int32_t launch_finalize(const smc_adam_args* adam, unsigned grid, const void* grads, int64_t n_params,
                        hipStream_t s) {
  hipLaunchKernelGGL(finalize_kernel<Real>, dim3(1), dim3(kNetThreads), 0, s, adam->norm_partials,
                     static_cast<int64_t>(grid), static_cast<const Real*>(grads), n_params, adam->step,
                     static_cast<Real*>(adam->grad_norm), static_cast<Real*>(adam->loss));
  return check_launch("cvnn finalize_kernel");
}

bool layers_valid(const smc_cvnn_layer* layers, int32_t n_layers, int64_t n_params) {
  if (!layers || n_layers <= 0 || n_layers > kMaxLayers) return false;
  for (int l = 0; l < n_layers; ++l) {
    const smc_cvnn_layer& ly = layers[l];
    if (ly.in_features <= 0 || ly.out_features <= 0) return false;
    if (l > 0 && ly.in_features != layers[l - 1].out_features) return false;
    if (ly.activation < SMC_ACT_NONE || ly.activation > SMC_ACT_ZRELU) return false;
    const int64_t w = static_cast<int64_t>(ly.in_features) * ly.out_features;
    if (ly.w_re < 0 || ly.w_im < 0 || ly.w_re + w > n_params || ly.w_im + w > n_params) return false;
    for (int64_t o : {ly.b_re, ly.b_im})
      if (o >= 0 && o + ly.out_features > n_params) return false;
    if (ly.activation == SMC_ACT_MODRELU && (ly.act_bias < 0 || ly.act_bias + ly.out_features > n_params))
      return false;
  }
  return true;
}

int32_t plan_rows(const smc_cvnn_layer* layers, int32_t n_layers, int32_t dtype, int64_t batch, int32_t* rows,
                  int64_t* blocks, size_t* lds) {
  const LdsPlan pl = plan_lds(layers, n_layers);
  const size_t elem = dtype == SMC_DTYPE_F64 ? 8 : 4;
  int r = 16;
  while (r > 1 && static_cast<size_t>(pl.per_row) * r * elem > kNetLdsBudget) r >>= 1;
  if (static_cast<size_t>(pl.per_row) * r * elem > kNetLdsBudget)
    return fail(SMC_ERR_INVALID_SHAPE, "cvnn: layer widths exceed the LDS budget");
  const int64_t n_blocks = (batch + r - 1) / r;
  *rows = r;
  *blocks = n_blocks < kMaxBlocks ? n_blocks : kMaxBlocks;
  *lds = static_cast<size_t>(pl.per_row) * r * elem;
  return SMC_OK;
}

template <typename Real, int R>
int32_t launch_fwd_bwd_r(const NetArgs& a, unsigned grid, size_t lds, hipStream_t s) {
  auto kernel = forward_backward_kernel<Real, R>;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          static_cast<int>(lds)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "cvnn forward_backward_kernel: cannot raise the dynamic LDS limit");
  }
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kNetThreads), lds, s, a);
  return SMC_OK;
}

template <typename Real>
int32_t launch_fwd_bwd(const NetArgs& a, unsigned grid, size_t lds, hipStream_t s) {
  switch (a.rows) {
    case 16: return launch_fwd_bwd_r<Real, 16>(a, grid, lds, s);
    case 8: return launch_fwd_bwd_r<Real, 8>(a, grid, lds, s);
    case 4: return launch_fwd_bwd_r<Real, 4>(a, grid, lds, s);
    case 2: return launch_fwd_bwd_r<Real, 2>(a, grid, lds, s);
    default: return launch_fwd_bwd_r<Real, 1>(a, grid, lds, s);
  }
}

}  // namespace
}  // namespace smc

using namespace smc;

#pragma GCC visibility push(default)
extern "C" {

int32_t smc_cvnn_plan(const smc_cvnn_layer* layers, int32_t n_layers, int32_t dtype, int64_t batch,
                      int64_t* partial_blocks) {
  if (!partial_blocks || batch <= 0 || (dtype != SMC_DTYPE_F32 && dtype != SMC_DTYPE_F64))
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_cvnn_plan: bad argument");
  if (!layers || n_layers <= 0 || n_layers > kMaxLayers)
    return fail(SMC_ERR_INVALID_SHAPE, "smc_cvnn_plan: 1..SMC_CVNN_MAX_LAYERS layers");
  int32_t rows;
  size_t lds;
  return plan_rows(layers, n_layers, dtype, batch, &rows, partial_blocks, &lds);
}

int32_t smc_cvnn_forward_backward(const smc_cvnn_layer* layers, int32_t n_layers, int32_t dtype, const void* params,
                                  int64_t n_params, const void* input_re, const void* input_im,
                                  const void* targets, int64_t batch, void* partials, int64_t partial_blocks,
                                  void* stream) {
  if (!params || !input_re || !targets || !partials || batch <= 0 ||
      (dtype != SMC_DTYPE_F32 && dtype != SMC_DTYPE_F64))
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_cvnn_forward_backward: bad argument");
  if (!layers_valid(layers, n_layers, n_params))
    return fail(SMC_ERR_INVALID_SHAPE, "smc_cvnn_forward_backward: inconsistent layer table");
  int32_t rows;
  int64_t blocks;
  size_t lds;
  const int32_t rc = plan_rows(layers, n_layers, dtype, batch, &rows, &blocks, &lds);
  if (rc != SMC_OK) return rc;
  if (partial_blocks != blocks) return fail(SMC_ERR_INVALID_SHAPE, "smc_cvnn_forward_backward: partial_blocks != plan");
  NetArgs a{};
  a.n_layers = n_layers;
  for (int l = 0; l < n_layers; ++l) a.layer[l] = layers[l];
  a.rows = rows;
  a.batch = batch;
  a.n_params = n_params;
  a.out_features = layers[n_layers - 1].out_features;
  a.params = params;
  a.input_re = input_re;
  a.input_im = input_im;
  a.targets = targets;
  a.partials = partials;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const int32_t lrc = dtype == SMC_DTYPE_F32 ? launch_fwd_bwd<float>(a, static_cast<unsigned>(blocks), lds, s)
                                             : launch_fwd_bwd<double>(a, static_cast<unsigned>(blocks), lds, s);
  if (lrc != SMC_OK) return lrc;
  return check_launch("cvnn forward_backward_kernel");
}

static AdamArgs to_adam(const smc_adam_args* ad, int64_t n_params, unsigned grid) {
  AdamArgs a{};
  a.params = ad->params;
  a.exp_avg = ad->exp_avg;
  a.exp_avg_sq = ad->exp_avg_sq;
  a.step = ad->step;
  a.lr = ad->lr;
  a.beta1 = ad->beta1;
  a.beta2 = ad->beta2;
  a.eps = ad->eps;
  a.weight_decay = ad->weight_decay;
  a.norm_partials = ad->norm_partials;
  if (ad->pack) a.pack = *ad->pack;  // else n_layers = 0
  a.norm_slots = smc_adam_norm_partials(n_params);
  a.grad_norm = ad->grad_norm;
  a.loss = ad->loss;
  a.fuse_final = grid <= kFuseFinalizeMaxBlocks ? 1 : 0;
  return a;
}

static bool adam_valid(const smc_adam_args* ad) {
  return ad->params && ad->exp_avg && ad->exp_avg_sq && ad->step && ad->norm_partials && ad->grad_norm &&
         ad->loss && ad->lr > 0.0 && ad->beta1 >= 0.0 && ad->beta1 < 1.0 && ad->beta2 >= 0.0 && ad->beta2 < 1.0;
}

// g^2 partials of reduce_kernel (one per 64 gradient entries; adam_kernel's fewer) + the arrival counter of the
// fused finalize (zero before the first call; the last workgroup leaves it zero)
static int64_t reduce_blocks(int64_t n_params) { return (n_params + 1 + kReduceCols - 1) / kReduceCols; }
int64_t smc_adam_norm_partials(int64_t n_params) { return reduce_blocks(n_params) + 1; }

int32_t smc_cvnn_reduce_grads(int32_t dtype, const void* partials, int64_t partial_blocks, int64_t n_params,
                              void* grads, const smc_adam_args* adam, void* stream) {
  if (!partials || !grads || partial_blocks <= 0 || n_params <= 0 ||
      (dtype != SMC_DTYPE_F32 && dtype != SMC_DTYPE_F64))
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_cvnn_reduce_grads: bad argument");
  if (adam && !adam_valid(adam)) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_cvnn_reduce_grads: bad Adam arguments");
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned grid = static_cast<unsigned>(reduce_blocks(n_params));  // 64 entries per block
  const AdamArgs ad = adam ? to_adam(adam, n_params, grid) : AdamArgs{};
  if (dtype == SMC_DTYPE_F32) {
    if (adam)
      hipLaunchKernelGGL((reduce_kernel<float, true>), dim3(grid), dim3(kNetThreads), 0, s,
                         static_cast<const float*>(partials), partial_blocks, n_params, static_cast<float*>(grads), ad);
    else
      hipLaunchKernelGGL((reduce_kernel<float, false>), dim3(grid), dim3(kNetThreads), 0, s,
                         static_cast<const float*>(partials), partial_blocks, n_params, static_cast<float*>(grads), ad);
  } else {
    if (adam)
      hipLaunchKernelGGL((reduce_kernel<double, true>), dim3(grid), dim3(kNetThreads), 0, s,
                         static_cast<const double*>(partials), partial_blocks, n_params, static_cast<double*>(grads), ad);
    else
      hipLaunchKernelGGL((reduce_kernel<double, false>), dim3(grid), dim3(kNetThreads), 0, s,
                         static_cast<const double*>(partials), partial_blocks, n_params, static_cast<double*>(grads), ad);
  }
  const int32_t rc = check_launch("cvnn reduce_kernel");
  if (rc != SMC_OK || !adam || ad.fuse_final) return rc;
  return dtype == SMC_DTYPE_F32 ? launch_finalize<float>(adam, grid, grads, n_params, s)
                                : launch_finalize<double>(adam, grid, grads, n_params, s);
}

int32_t smc_adam_step(int32_t dtype, int64_t n_params, const void* grads, const smc_adam_args* adam, void* stream) {
  if (!grads || !adam || n_params <= 0 || (dtype != SMC_DTYPE_F32 && dtype != SMC_DTYPE_F64))
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_adam_step: bad argument");
  if (!adam_valid(adam)) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_adam_step: bad Adam arguments");
  const hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned grid = static_cast<unsigned>((n_params + kNetThreads - 1) / kNetThreads);
  const AdamArgs ad = to_adam(adam, n_params, grid);
  if (dtype == SMC_DTYPE_F32)
    hipLaunchKernelGGL(adam_kernel<float>, dim3(grid), dim3(kNetThreads), 0, s, static_cast<const float*>(grads),
                       n_params, ad);
  else
    hipLaunchKernelGGL(adam_kernel<double>, dim3(grid), dim3(kNetThreads), 0, s, static_cast<const double*>(grads),
                       n_params, ad);
  const int32_t rc = check_launch("adam_kernel");
  if (rc != SMC_OK || ad.fuse_final) return rc;
  return dtype == SMC_DTYPE_F32 ? launch_finalize<float>(adam, grid, grads, n_params, s)
                                : launch_finalize<double>(adam, grid, grads, n_params, s);
}

}  // extern "C"
#pragma GCC visibility pop
