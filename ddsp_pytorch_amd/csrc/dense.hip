// The decoder's control network for a few frames at a time (the realtime stream: 4 frames per
// 1024-sample call, BASELINE.json config 3).  ddsp/core.py:122-129 builds every MLP block as
// Linear -> LayerNorm -> LeakyReLU; decoder.py:43-68 chains three such MLPs, the GRU input
// projection, the output MLP and the two projections (decoder.py:107-114).  At 4 rows each of
// those ~25 torch ops is a launch-bound kernel of ~4-6 us (rocprofv3, 190 us per call).
//
// Here one launch computes one Linear for every row, with the previous block's LayerNorm +
// LeakyReLU (and a K=1 first Linear, the loudness normalisation, the concatenations of
// decoder.py:49,68) folded into how it reads its inputs:
//   a[r, :] = concat_s act_s(x_s[r, :])                     (built in LDS, rows x K)
//   y[r, n] = sum_k W[n, k] a[r, k] + b[n]                   (one wave per output row of W)
// act_s: x' = x * scale + shift; if w1: x'' = w1[c] * x' + b1[c] (c < width; x' is one value per
// row); if gamma: leaky_relu(layer_norm(x'') * gamma + beta, 0.01) with torch's eps 1e-5 and
// biased variance.  W rows are streamed once per launch with coalesced loads; each workgroup
// recomputes the (tiny) activations.  Up to kMaxProblems independent Linears share a launch
// (blockIdx.y), e.g. the f0 and loudness MLPs, or the harmonic and noise projections.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"

namespace ddsp {
namespace {

constexpr int kDenseNT = 512;      // 8 waves
constexpr int kOutPerWave = 1;     // output features per wave
constexpr int kOutPerWG = (kDenseNT / 64) * kOutPerWave;
constexpr int kMaxRows = 8;
constexpr int kKL = 17;            // K <= 64 * kKL per lane-strided row (1088: the GRU input's 1024)

struct DenseArgs {
  ddsp_hip_dense_problem p[DDSP_HIP_DENSE_MAX_PROBLEMS];
  int rows;
};

// Sum over the wave, returned uniform: DPP quad permutes for lane distances 1 and 2,
// ds_swizzle xor for 4, 8, 16 (within each half), then the two halves by readlane — no
// ds_bpermute address arithmetic, no LDS round trip (the 6-step __shfl_xor tree cost ~3 us of
// a 10 us launch here).
__device__ __forceinline__ float wave_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));  // quad_perm 1,0,3,2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));  // quad_perm 2,3,0,1
  v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x101F));  // xor 4
  v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x201F));  // xor 8
  v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));  // xor 16
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
         __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
}

// At 4 rows everything here is latency: every global load a wave needs is issued before the
// first use (W rows straight into registers at kernel entry, under the activation prologue),
// and the cross-lane sums avoid ds_bpermute.
__global__ void __launch_bounds__(kDenseNT) dense_rows_kernel(DenseArgs args) {
  extern __shared__ float act[];  // [rows][K]
  const ddsp_hip_dense_problem& P = args.p[blockIdx.y];
  const int n0 = blockIdx.x * kOutPerWG;
  if (n0 >= P.out_features) return;
  const int rows = args.rows, lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: scalar row bases
  int K = 0;
  for (int s = 0; s < P.n_inputs; ++s) K += (int)P.inputs[s].width;

  // ---- W rows of this wave's outputs into registers ----
  float wreg[kOutPerWave][kKL];
  // (loads branch-free: a clamped address and a select; chunk guards j < nK are wave-uniform)
  const int nK = (K + 63) >> 6;
#pragma unroll
  for (int i = 0; i < kOutPerWave; ++i) {
    const int n = min(n0 + wave * kOutPerWave + i, (int)P.out_features - 1);
    const float* wr = P.weight + (int64_t)n * K;
#pragma unroll
    for (int j = 0; j < kKL; ++j) {
      const unsigned k = lane + 64 * j;
      const float w = wr[min(k, (unsigned)K - 1u)];  // unconditional: every address is valid
      wreg[i][j] = k < (unsigned)K ? w : 0.0f;
    }
  }

  // ---- activations: wave w builds (segment, row) pairs w, w+4, ... ----
  int col0 = 0;
  for (int s = 0; s < P.n_inputs; ++s) {
    const ddsp_hip_dense_input& in = P.inputs[s];
    const int width = (int)in.width;
    for (int r = wave; r < rows; r += kDenseNT / 64) {
      const float* xr = in.x + (int64_t)r * in.ld;
      float* ar = act + (int64_t)r * K + col0;
      const int nC = (width + 63) >> 6;
      float v[kKL], gm[kKL], bt[kKL];
      if (in.gamma) {  // issued with the inputs, before the first reduction
#pragma unroll
        for (int j = 0; j < kKL; ++j) {
          const int cc = min(lane + 64 * j, width - 1);
          gm[j] = in.gamma[cc];
          bt[j] = in.beta[cc];
        }
      }
      float sum = 0.0f;
      if (in.w1) {
        const float xs = fmaf(xr[0], in.scale, in.shift);
        if (in.x_copy && blockIdx.x == 0 && lane == 0) in.x_copy[r] = xs;
#pragma unroll
        for (int j = 0; j < kKL; ++j) {
          const int cc = min(lane + 64 * j, width - 1);
          const float t = fmaf(in.w1[cc], xs, in.b1[cc]);
          v[j] = lane + 64 * j < width ? t : 0.0f;
          sum += v[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < kKL; ++j) {
          const int cc = min(lane + 64 * j, width - 1);
          const float t = fmaf(xr[cc], in.scale, in.shift);
          v[j] = lane + 64 * j < width ? t : 0.0f;
          sum += v[j];
        }
      }
      if (in.gamma) {  // LayerNorm (two-pass, biased variance) + LeakyReLU over this segment
        const float mean = wave_sum(sum) / (float)width;
        float sq = 0.0f;
#pragma unroll
        for (int j = 0; j < kKL; ++j) {
          const float d = lane + 64 * j < width ? v[j] - mean : 0.0f;
          sq += d * d;
        }
        const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)width + 1e-5f);
#pragma unroll
        for (int j = 0; j < kKL; ++j) {
          const float t = (v[j] - mean) * rstd * gm[j] + bt[j];
          v[j] = t >= 0.0f ? t : 0.01f * t;
        }
      }
#pragma unroll
      for (int j = 0; j < kKL; ++j)
        if (j < nC && lane + 64 * j < width) ar[lane + 64 * j] = v[j];
    }
    col0 += width;
  }
  __syncthreads();

  // ---- GEMV from registers x LDS, then step-major wave sums ----
  float acc[kOutPerWave][kMaxRows];
#pragma unroll
  for (int i = 0; i < kOutPerWave; ++i)
#pragma unroll
    for (int r = 0; r < kMaxRows; ++r) acc[i][r] = 0.0f;
#pragma unroll
  for (int j = 0; j < kKL; ++j) {
    if (j < nK) {  // wave-uniform; past K the weights are 0 and the activation index is clamped
      const int k = min(lane + 64 * j, K - 1);
#pragma unroll
      for (int r = 0; r < kMaxRows; ++r) {
        if (r < rows) {
          const float a = act[r * K + k];
#pragma unroll
          for (int i = 0; i < kOutPerWave; ++i) acc[i][r] = fmaf(wreg[i][j], a, acc[i][r]);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kOutPerWave; ++i)
#pragma unroll
    for (int r = 0; r < kMaxRows; ++r)
      if (r < rows) acc[i][r] = wave_sum(acc[i][r]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < kOutPerWave; ++i) {
      const int n = n0 + wave * kOutPerWave + i;
      if (n < P.out_features) {
        const float bn = P.bias ? P.bias[n] : 0.0f;
#pragma unroll
        for (int r = 0; r < kMaxRows; ++r)
          if (r < rows) P.y[(int64_t)r * P.ldy + n] = acc[i][r] + bn;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// The decoder's MLP blocks at full batch (ddsp/core.py:122-129: Linear -> LayerNorm -> LeakyReLU):
// the Linear stays a hipBLASLt GEMM, and LayerNorm + LeakyReLU run as ONE pass over its output
// (torch runs two: 18 + 11 us per [12800, 512] layer at config 2), one wave per row, the row in
// registers (cols/64 values per lane), mean and biased variance by two wave sums (two-pass, as
// accurate as torch's Welford), eps inside the root as torch does.  With w1/b1 the block's Linear
// has one input feature (the f0 / loudness MLPs' first layer, decoder.py:25-30): h = x w1 + b1 is
// formed on the fly (product, then bias: the GEMM's two roundings).  y may be a column slice of a
// wider buffer (y_ld), so the f0 and loudness MLPs write straight into the GRU's input
// concatenation (decoder.py:46-49) with no torch.cat.
template <int V4>  // float4 per lane: cols = 256 * V4
__global__ void __launch_bounds__(256) ln_leaky_kernel(const float* __restrict__ x, int64_t x_ld,
                                                       const float* __restrict__ w1, const float* __restrict__ b1,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, float slope, float* __restrict__ y, int64_t y_ld,
                                                       int64_t rows) {
  constexpr int C = 256 * V4;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  float4 v[V4];
  if (w1) {
    const float xv = x[row * x_ld];
#pragma unroll
    for (int i = 0; i < V4; ++i) {
      const float4 w = reinterpret_cast<const float4*>(w1)[lane + 64 * i];
      const float4 b = reinterpret_cast<const float4*>(b1)[lane + 64 * i];
      v[i] = make_float4(xv * w.x + b.x, xv * w.y + b.y, xv * w.z + b.z, xv * w.w + b.w);
    }
  } else {
#pragma unroll
    for (int i = 0; i < V4; ++i) v[i] = reinterpret_cast<const float4*>(x + row * x_ld)[lane + 64 * i];
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < V4; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = wave_sum(s) * (1.0f / (float)C);
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
    q += (a * a + b * b) + (c * c + d * d);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) * (1.0f / (float)C) + eps);
  float4* yr = reinterpret_cast<float4*>(y + row * y_ld);
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    const float4 g = reinterpret_cast<const float4*>(gamma)[lane + 64 * i];
    const float4 bt = reinterpret_cast<const float4*>(beta)[lane + 64 * i];
    float o[4] = {(v[i].x - mean) * rstd * g.x + bt.x, (v[i].y - mean) * rstd * g.y + bt.y,
                  (v[i].z - mean) * rstd * g.z + bt.z, (v[i].w - mean) * rstd * g.w + bt.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = o[e] >= 0.0f ? o[e] : o[e] * slope;
    yr[lane + 64 * i] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// Backward of ln_leaky_kernel (training: the MLP blocks' LayerNorm + LeakyReLU, ddsp/core.py:122-129, under
// autograd).  Per row, from the saved pre-activation x: mean / rstd as the forward forms them, n = (x - mean) rstd,
// z = n gamma + beta (the forward's expression, so the LeakyReLU's branch is the forward's), dz = dy (z > 0 ? 1 :
// slope) (torch's leaky_relu_backward), dn = dz gamma, dx = rstd (dn - mean(dn) - n mean(dn n)) (torch's
// layer_norm backward for the biased variance).  One wave per row over a fixed grid (rows w, w + 4 gridDim, ...), so
// each lane keeps its columns' dgamma = sum dz n and dbeta = sum dz in registers; the workgroup's 4 waves are summed
// in LDS into one partial per workgroup, and ln_leaky_bwd_sum_kernel adds the partials in workgroup order
// (deterministic, no atomics).
constexpr int kLnBwdGrid = 256;
template <int V4>
__global__ void __launch_bounds__(256) ln_leaky_bwd_kernel(const float* __restrict__ x, int64_t x_ld,
                                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                                           float eps, float slope, const float* __restrict__ dy,
                                                           int64_t dy_ld, float* __restrict__ dx, int64_t dx_ld,
                                                           float* __restrict__ part, int64_t rows) {
  constexpr int C = 256 * V4;
  __shared__ float4 red[4][2][64 * V4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float4 gm[V4], bt[V4], dgs[V4], dbs[V4];
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    gm[i] = reinterpret_cast<const float4*>(gamma)[lane + 64 * i];
    bt[i] = reinterpret_cast<const float4*>(beta)[lane + 64 * i];
    dgs[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    dbs[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < rows; row += (int64_t)gridDim.x * 4) {
    float4 v[V4], d[V4];
#pragma unroll
    for (int i = 0; i < V4; ++i) {
      v[i] = reinterpret_cast<const float4*>(x + row * x_ld)[lane + 64 * i];
      d[i] = reinterpret_cast<const float4*>(dy + row * dy_ld)[lane + 64 * i];
    }
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < V4; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    const float mean = wave_sum(s) * (1.0f / (float)C);
    float q = 0.0f;
#pragma unroll
    for (int i = 0; i < V4; ++i) {
      const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, e = v[i].w - mean;
      q += (a * a + b * b) + (c * c + e * e);
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) * (1.0f / (float)C) + eps);
    float nn[4 * V4], dn[4 * V4];
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int i = 0; i < V4; ++i) {
      const float vv[4] = {v[i].x, v[i].y, v[i].z, v[i].w}, dd[4] = {d[i].x, d[i].y, d[i].z, d[i].w};
      const float gg[4] = {gm[i].x, gm[i].y, gm[i].z, gm[i].w}, bb[4] = {bt[i].x, bt[i].y, bt[i].z, bt[i].w};
      float dz[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float n = (vv[e] - mean) * rstd;
        const float z = n * gg[e] + bb[e];
        dz[e] = z > 0.0f ? dd[e] : dd[e] * slope;
        nn[4 * i + e] = n;
        dn[4 * i + e] = dz[e] * gg[e];
        s1 += dn[4 * i + e];
        s2 += dn[4 * i + e] * n;
      }
      dgs[i] = make_float4(dgs[i].x + dz[0] * nn[4 * i], dgs[i].y + dz[1] * nn[4 * i + 1],
                           dgs[i].z + dz[2] * nn[4 * i + 2], dgs[i].w + dz[3] * nn[4 * i + 3]);
      dbs[i] = make_float4(dbs[i].x + dz[0], dbs[i].y + dz[1], dbs[i].z + dz[2], dbs[i].w + dz[3]);
    }
    const float m1 = wave_sum(s1) * (1.0f / (float)C), m2 = wave_sum(s2) * (1.0f / (float)C);
    float4* dr = reinterpret_cast<float4*>(dx + row * dx_ld);
#pragma unroll
    for (int i = 0; i < V4; ++i)
      dr[lane + 64 * i] = make_float4(rstd * (dn[4 * i] - m1 - nn[4 * i] * m2), rstd * (dn[4 * i + 1] - m1 - nn[4 * i + 1] * m2),
                                      rstd * (dn[4 * i + 2] - m1 - nn[4 * i + 2] * m2),
                                      rstd * (dn[4 * i + 3] - m1 - nn[4 * i + 3] * m2));
  }
  if (!part) return;
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    red[w][0][lane + 64 * i] = dgs[i];
    red[w][1][lane + 64 * i] = dbs[i];
  }
  __syncthreads();
  // thread t sums the 4 waves for float4 slot t of [dgamma | dbeta] (2 * 64 V4 slots)
  for (int t = threadIdx.x; t < 2 * 64 * V4; t += 256) {
    const int h = t / (64 * V4), k = t - h * (64 * V4);
    float4 a = red[0][h][k];
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) {
      const float4 b = red[ww][h][k];
      a = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
    reinterpret_cast<float4*>(part + (int64_t)blockIdx.x * 2 * C + h * C)[k] = a;
  }
}

// [dgamma | dbeta][c] = sum over the workgroups' partials: a workgroup per 64 columns, its 4 waves summing the
// partials j, j + 4, ... (coalesced over the 64 columns), then the 4 wave sums in wave order (deterministic)
__global__ void __launch_bounds__(256) ln_leaky_bwd_sum_kernel(const float* __restrict__ part, int nparts, int C,
                                                               float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float a = 0.0f;
  if (c < 2 * C) {
#pragma unroll 8
    for (int b = w; b < nparts; b += 4) a += part[(int64_t)b * 2 * C + c];
  }
  red[w][lane] = a;
  __syncthreads();
  if (w != 0 || c >= 2 * C) return;
  const float s = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
  if (c < C) {
    if (dgamma) dgamma[c] = s;
  } else if (dbeta) {
    dbeta[c - C] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// One whole MLP block at full batch (ddsp/core.py:122-129): y = LeakyReLU(LayerNorm(x W^T + b)) for
// 512 output features, the Linear on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact fp32
// products and sums) and LayerNorm + LeakyReLU in the epilogue, so the block's [rows, 512] result is
// written once (hipBLASLt's GEMM wrote it, then LayerNorm and LeakyReLU re-read and re-wrote it).
// A workgroup owns 64 full rows (LayerNorm needs whole rows), its 8 waves 64 output columns each as a
// 4 x 4 grid of 16 x 16 MFMA tiles.  x and W stream through ONE LDS stage of K = 32 per step: the
// next step's operands are loaded into registers at the top of a step and written to LDS after its
// 128 MFMAs per wave, so each load's latency hides under a whole step of matrix work (a 16-wide,
// double-buffered LDS stage left the loads exposed: 103 us per config-2 block, against 55 us of
// MFMA issue).  Within a step lane l supplies k = 16 h + 4 (l >> 4) + s at sub-step (h, s) for both
// operands (one ds_read_b128 per operand tile per half), so every product pairs x[r][k] with W[c][k].
// kVec: 4 = 16-byte loads (x and W rows 16-B aligned, K % 4 == 0); 2 = 8-byte loads (rows 8-B aligned,
// K % 4 == 0: the out_mlp's W, 514 floats a row); 1 = scalar loads.  e0/e1
// (optional): per-row scalars with weight columns K and K + 1 — the decoder's out_mlp input
// [gru_out, f0, loudness] (decoder.py:68) without materialising the concatenation.
constexpr int kMlpN = 512;          // output features (8 waves x 64)
constexpr int kMlpRows = 64;        // rows per workgroup
constexpr int kMlpKC = 32;          // K per LDS stage
constexpr int kMlpLd = kMlpKC + 4;  // LDS row stride (floats): 16-B aligned rows, banks spread

// The block's epilogue (both forms below): bias, the out_mlp's two extra input columns, LayerNorm (two-pass
// mean / biased variance over the row, reduced across the 8 waves in LDS) and LeakyReLU, one store per value.
__device__ __forceinline__ void mlp_epilogue(f32x4_t (&acc)[4][4], int64_t r0, int K, const float* __restrict__ w,
                                             int64_t w_ld, const float* __restrict__ bias,
                                             const float* __restrict__ e0, const float* __restrict__ e1, int64_t e_ld,
                                             const float* __restrict__ gamma, const float* __restrict__ beta,
                                             float eps, float slope, float* __restrict__ y, int64_t y_ld, int64_t R,
                                             float (*red)[kMlpRows], float* stat) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int q = lane >> 4, l16 = lane & 15;
  // epilogue: acc[i][j][e] is row 16 i + 4 q + e, column 64 wv + 16 j + l16
  float cb[4], cw0[4], cw1[4], cg[4], cbt[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 64 * wv + 16 * j + l16;
    cb[j] = bias[col];
    cw0[j] = e0 ? w[(int64_t)col * w_ld + K] : 0.0f;
    cw1[j] = e1 ? w[(int64_t)col * w_ld + K + 1] : 0.0f;
    cg[j] = gamma[col];
    cbt[j] = beta[col];
  }
  float v[4][4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t row = r0 + 16 * i + 4 * q + e;
      const bool ok = row < R;
      const float x0 = (e0 && ok) ? e0[row * e_ld] : 0.0f, x1 = (e1 && ok) ? e1[row * e_ld] : 0.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float h = acc[i][j][e] + cb[j];
        if (e0) h += x0 * cw0[j];
        if (e1) h += x1 * cw1[j];
        v[i][j][e] = h;
      }
    }
  // row means, then the biased variance about them (two passes, as accurate as torch's Welford)
  auto row_reduce = [&](auto&& term) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float sum = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) sum += term(i, j, e);
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);  // the 16 lanes of one row
        if (l16 == 0) red[wv][16 * i + 4 * q + e] = sum;
      }
    __syncthreads();
    if (t < kMlpRows) {
      float sum = 0.0f;
#pragma unroll
      for (int k = 0; k < 8; ++k) sum += red[k][t];
      stat[t] = sum * (1.0f / (float)kMlpN);
    }
    __syncthreads();
  };
  row_reduce([&](int i, int j, int e) { return v[i][j][e]; });
  float mean[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) mean[i][e] = stat[16 * i + 4 * q + e];
  row_reduce([&](int i, int j, int e) {
    const float d = v[i][j][e] - mean[i][e];
    return d * d;
  });
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t row = r0 + 16 * i + 4 * q + e;
      if (row >= R) continue;
      const float rstd = 1.0f / sqrtf(stat[16 * i + 4 * q + e] + eps);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float o = (v[i][j][e] - mean[i][e]) * rstd * cg[j] + cbt[j];
        o = o >= 0.0f ? o : o * slope;
        y[row * y_ld + 64 * wv + 16 * j + l16] = o;
      }
    }
}

template <int kVec>
__global__ void __launch_bounds__(512) mlp_block_kernel(
    const float* __restrict__ x, int64_t x_ld, int K, const float* __restrict__ w, int64_t w_ld,
    const float* __restrict__ bias, const float* __restrict__ e0, const float* __restrict__ e1, int64_t e_ld,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float slope, float* __restrict__ y,
    int64_t y_ld, int64_t R) {
  __shared__ __attribute__((aligned(16))) float As[kMlpRows * kMlpLd];
  __shared__ __attribute__((aligned(16))) float Bs[kMlpN * kMlpLd];
  __shared__ float red[8][kMlpRows];
  __shared__ float stat[kMlpRows];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int q = lane >> 4, l16 = lane & 15;
  const int64_t r0 = (int64_t)blockIdx.x * kMlpRows;
  const int nc = (K + kMlpKC - 1) / kMlpKC;
  // per step: x tile 64 x 32 (one float4 per thread), W tile 512 x 32 (eight float4 per thread);
  // float4 f of the tile is (row f >> 3, k 4 (f & 7))
  float4 sa, sb[8];
  auto ld4 = [&](const float* row, int k) -> float4 {  // row[k .. k+3], zero past K
    if constexpr (kVec == 4) {
      return k < K ? *reinterpret_cast<const float4*>(row + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else if constexpr (kVec == 2) {
      if (k >= K) return make_float4(0.f, 0.f, 0.f, 0.f);
      const float2 a = *reinterpret_cast<const float2*>(row + k), b = *reinterpret_cast<const float2*>(row + k + 2);
      return make_float4(a.x, a.y, b.x, b.y);
    } else {
      return make_float4(k < K ? row[k] : 0.f, k + 1 < K ? row[k + 1] : 0.f, k + 2 < K ? row[k + 2] : 0.f,
                         k + 3 < K ? row[k + 3] : 0.f);
    }
  };
  auto load = [&](int c) {
    const int k0 = c * kMlpKC;
    {
      const int row = t >> 3, k = k0 + 4 * (t & 7);
      const int64_t rr = r0 + row < R ? r0 + row : R - 1;  // rows >= R: loaded, never stored
      sa = ld4(x + rr * x_ld, k);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int f = t + 512 * i, col = f >> 3, k = k0 + 4 * (f & 7);
      sb[i] = ld4(w + (int64_t)col * w_ld, k);
    }
  };
  auto store = [&]() {
    *reinterpret_cast<float4*>(&As[(t >> 3) * kMlpLd + 4 * (t & 7)]) = sa;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int f = t + 512 * i;
      *reinterpret_cast<float4*>(&Bs[(f >> 3) * kMlpLd + 4 * (f & 7)]) = sb[i];
    }
  };
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int c = 0; c < nc; ++c) {
    __syncthreads();  // every wave is done reading the previous step's stage
    store();
    __syncthreads();
    if (c + 1 < nc) load(c + 1);  // in flight under this step's MFMAs
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float4 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = *reinterpret_cast<const float4*>(&As[(16 * i + l16) * kMlpLd + 16 * h + 4 * q]);
        bf[i] = *reinterpret_cast<const float4*>(&Bs[(64 * wv + 16 * i + l16) * kMlpLd + 16 * h + 4 * q]);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a = s == 0 ? af[i].x : s == 1 ? af[i].y : s == 2 ? af[i].z : af[i].w;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float b = s == 0 ? bf[j].x : s == 1 ? bf[j].y : s == 2 ? bf[j].z : bf[j].w;
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i][j], 0, 0, 0);
          }
        }
      }
    }
  }
  mlp_epilogue(acc, r0, K, w, w_ld, bias, e0, e1, e_ld, gamma, beta, eps, slope, y, y_ld, R, red, stat);
}

// The same block with the x tile RESIDENT in LDS and W streamed straight into MFMA operand registers (the
// decoder's blocks: K = 512).  Why: in the staged form above every K step is a pair of workgroup barriers
// around one LDS stage that all 8 waves fill and then read, so the matrix pipe idles for the barrier, the
// LDS writes and the first reads of every step (89 us per config-2 block against ~55 us of MFMA issue).
// Here the workgroup's 64 x K slice of x is loaded into LDS once (133 KB at K = 512, rows padded to
// K + 8 floats: the 16-lane groups of a ds_read_b128 then hit 16 distinct bank quads), and W needs no
// LDS at all — wave wv alone uses output columns [64 wv, 64 wv + 64), so each lane loads its B fragment
// (column 64 wv + 16 j + l16, k = 16 h + 4 q .. + 3: one float4 per tile and 16-wide K chunk h) from
// global memory kP chunks ahead of its use into a register ring.  The main loop has no barrier: each wave
// runs 4 LDS reads + 4 global loads + 64 MFMAs per chunk on its own.  Same operands per MFMA and the same
// k order as the staged form (k = 16 h + 4 q + s at sub-step s), so the results are identical bit for bit.
constexpr int kMlpResK = 512;
constexpr int kMlpResLd = kMlpResK + 8;
template <int kP>
__global__ void __launch_bounds__(512) mlp_block_res_kernel(
    const float* __restrict__ x, int64_t x_ld, const float* __restrict__ w, int64_t w_ld,
    const float* __restrict__ bias, const float* __restrict__ e0, const float* __restrict__ e1, int64_t e_ld,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float slope, float* __restrict__ y,
    int64_t y_ld, int64_t R) {
  constexpr int K = kMlpResK, NH = K / 16;
  static_assert(NH % kP == 0, "ring");
  __shared__ __attribute__((aligned(16))) float xs[kMlpRows * kMlpResLd];
  __shared__ float red[8][kMlpRows];
  __shared__ float stat[kMlpRows];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int q = lane >> 4, l16 = lane & 15;
  const int64_t r0 = (int64_t)blockIdx.x * kMlpRows;
  // this lane's W fragment rows: column 64 wv + 16 j + l16, k offset 4 q
  const float* wl = w + (int64_t)(64 * wv + l16) * w_ld + 4 * q;
  const int64_t wj = 16 * w_ld;
  float4 wb[kP][4];
#pragma unroll
  for (int p = 0; p < kP; ++p)
#pragma unroll
    for (int j = 0; j < 4; ++j) wb[p][j] = *reinterpret_cast<const float4*>(wl + j * wj + 16 * p);
  // the x tile into LDS (rows >= R read row R - 1: loaded, never stored)
  {
    constexpr int kF4 = kMlpRows * K / 4 / 512;  // float4 per thread
    float4 v[kF4];
#pragma unroll
    for (int i = 0; i < kF4; ++i) {
      const int f = t + 512 * i, row = f / (K / 4), c4 = f - row * (K / 4);
      const int64_t rr = r0 + row < R ? r0 + row : R - 1;
      v[i] = *reinterpret_cast<const float4*>(x + rr * x_ld + 4 * c4);
    }
#pragma unroll
    for (int i = 0; i < kF4; ++i) {
      const int f = t + 512 * i, row = f / (K / 4), c4 = f - row * (K / 4);
      *reinterpret_cast<float4*>(&xs[row * kMlpResLd + 4 * c4]) = v[i];
    }
  }
  __syncthreads();
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  const float* xl = xs + l16 * kMlpResLd + 4 * q;
  for (int h0 = 0; h0 < NH; h0 += kP) {
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      const int h = h0 + p;
      float4 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const float4*>(xl + 16 * i * kMlpResLd + 16 * h);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a = s == 0 ? af[i].x : s == 1 ? af[i].y : s == 2 ? af[i].z : af[i].w;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float b = s == 0 ? wb[p][j].x : s == 1 ? wb[p][j].y : s == 2 ? wb[p][j].z : wb[p][j].w;
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i][j], 0, 0, 0);
          }
        }
      }
      // refill this ring slot with chunk h + kP (clamped: the last kP reloads re-read the final chunk, so
      // every iteration issues the same loads and the wait counts stay exact)
      const int hn = h + kP < NH ? h + kP : NH - 1;
#pragma unroll
      for (int j = 0; j < 4; ++j) wb[p][j] = *reinterpret_cast<const float4*>(wl + j * wj + 16 * hn);
      __builtin_amdgcn_sched_barrier(0);  // keep the refill here (the scheduler would sink it to the slot's use)
    }
  }
  mlp_epilogue(acc, r0, K, w, w_ld, bias, e0, e1, e_ld, gamma, beta, eps, slope, y, y_ld, R, red, stat);
}

// The decoder's blocks (K = 512) on the bf16 matrix cores with fp32 accuracy.  The f32-input MFMA runs at
// 1/16 of the bf16 rate, and the kernels above are bound by it (84-90 us per config-2 block: 74 TF on the
// 200 CUs a 12,800-row batch fills, at the clock MFMA-dense loops hold).  Here both operands are split
// exactly into three bf16 terms, v = hi + mid + lo (hi = v with its low 16 bits cleared, mid the same of
// v - hi, lo = v - hi - mid: each term exact, 8 significant bits apiece, together all 24 of the fp32
// significand), and each 16 x 16 x 32 product is the six MFMAs hi.hi, hi.mid, mid.hi, hi.lo, lo.hi, mid.mid
// — every bf16 x bf16 product is exact in fp32; the dropped mid.lo, lo.mid, lo.lo terms are < 2^-16 x 2^-8
// of the product: an fp32-accurate GEMM (not bit-identical to the f32 MFMA's fma chain) at 6/16 of its
// matrix time.  The split is VALU work, which the MFMAs leave free for 8 of every 16 issue cycles:
//   * x (shared by the 8 waves) is split ONCE per workgroup, a quarter of K (128) at a time, into three bf16
//     planes in LDS (48 KB per quarter, two quarters resident, 16-byte quads XOR-swizzled by row so that the
//     fragment reads and the split's writes are conflict-free); the next quarter's fp32 loads are in
//     flight during the current quarter's MFMAs; one barrier per quarter;
//   * W (each wave alone uses its 64 output columns) is split by its wave, streamed from global memory into
//     a register ring kP 32-wide chunks ahead of its use (no LDS).
// Fragments (v_mfma_f32_16x16x32_bf16): lane (q, l16) holds A[row l16][k = 8 q .. + 7] and
// B[k = 8 q .. + 7][col l16]; C/D as the f32 form (row 4 q + e, col l16), so the epilogue is shared.
// (split_bf16x3, u32x4_t and as_bf16x8: common.h)

constexpr int kBf3QK = 128;                     // K per quarter (LDS split stage)
constexpr int kBf3Plane = kMlpRows * kBf3QK;    // bf16 elements per plane (row-major, 256 B rows)

// kLN: the MLP block (512 outputs, LayerNorm + LeakyReLU epilogue); else a plain Linear, y = x W^T + b, over
// 512-column blocks of W (blockIdx.y), e.g. the GRU's input projection for every step (decoder.py:41).
// kW8: W rows only 8-byte aligned (the out_mlp's first Linear, 514 inputs: decoder.py:68) -> 8-byte loads.
template <int kP, int K, bool kLN, bool kW8 = false>
__global__ void __launch_bounds__(512) linear_bf3_kernel(
    const float* __restrict__ x, int64_t x_ld, const float* __restrict__ w, int64_t w_ld,
    const float* __restrict__ bias, const float* __restrict__ e0, const float* __restrict__ e1, int64_t e_ld,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float slope, float* __restrict__ y,
    int64_t y_ld, int64_t R) {
  constexpr int NQ = K / kBf3QK, NC = kBf3QK / 32;  // quarters; 32-wide chunks per quarter
  static_assert(K % kBf3QK == 0 && NQ >= 2, "K");
  static_assert((NQ * NC) % kP == 0 && NC % kP == 0, "ring");
  // [buffer][plane hi/mid/lo][row][128 k] bf16, quads (8 bf16) at position Q ^ (row & 15)
  __shared__ __attribute__((aligned(16))) uint32_t xs[2 * 3 * kBf3Plane / 2];
  __shared__ float red[8][kMlpRows];
  __shared__ float stat[kMlpRows];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int q = lane >> 4, l16 = lane & 15;
  const int64_t r0 = (int64_t)blockIdx.x * kMlpRows;
  if (!kLN) {  // this workgroup's 512 output columns
    w += (int64_t)blockIdx.y * kMlpN * w_ld;
    bias += blockIdx.y * kMlpN;
    y += blockIdx.y * kMlpN;
  }
  // W fragment of this lane: column 64 wv + 16 j + l16, k = 32 h + 8 q .. + 7 (two float4)
  const float* wl = w + (int64_t)(64 * wv + l16) * w_ld + 8 * q;
  const int64_t wj = 16 * w_ld;
  auto ldw = [](const float* p) -> float4 {
    if constexpr (kW8) {
      const float2 a = *reinterpret_cast<const float2*>(p), b = *reinterpret_cast<const float2*>(p + 2);
      return make_float4(a.x, a.y, b.x, b.y);
    } else {
      return *reinterpret_cast<const float4*>(p);
    }
  };
  float4 wb[kP][4][2];
#pragma unroll
  for (int p = 0; p < kP; ++p)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wb[p][j][0] = ldw(wl + j * wj + 32 * p);
      wb[p][j][1] = ldw(wl + j * wj + 32 * p + 4);
    }
  // split role: thread -> row t >> 3, k 16 (t & 7) .. + 15 of a quarter (quads Q = 2 (t & 7), + 1)
  const int srow = t >> 3, sq = 2 * (t & 7);
  const float* xsrc = x + (r0 + srow < R ? r0 + srow : R - 1) * x_ld + 8 * sq;  // rows >= R: never stored
  float4 xv[4];
  auto load_quarter = [&](int qt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) xv[i] = *reinterpret_cast<const float4*>(xsrc + kBf3QK * qt + 4 * i);
  };
  auto store_quarter = [&](int buf) {
    u32x4_t hq[2], mq[2], lq[2];
    split_bf16x3(xv[0], xv[1], hq[0], mq[0], lq[0]);
    split_bf16x3(xv[2], xv[3], hq[1], mq[1], lq[1]);
    uint32_t* base = xs + buf * (3 * kBf3Plane / 2) + srow * (kBf3QK / 2);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int pos = 4 * ((sq + e) ^ (srow & 15));  // uint32 offset of the quad
      *reinterpret_cast<u32x4_t*>(base + pos) = hq[e];
      *reinterpret_cast<u32x4_t*>(base + kBf3Plane / 2 + pos) = mq[e];
      *reinterpret_cast<u32x4_t*>(base + kBf3Plane + pos) = lq[e];
    }
  };
  load_quarter(0);
  store_quarter(0);
  load_quarter(1);
  store_quarter(1);
  load_quarter(2);  // in flight under quarter 0
  __syncthreads();
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  for (int qt = 0; qt < NQ; ++qt) {
    const uint32_t* xb = xs + (qt & 1) * (3 * kBf3Plane / 2) + l16 * (kBf3QK / 2);  // row 16 i + l16: row & 15 = l16
#pragma unroll
    for (int c0 = 0; c0 < NC; c0 += kP) {
#pragma unroll
      for (int p = 0; p < kP; ++p) {
        const int c = c0 + p, h = qt * NC + c;
        const int pos = 4 * ((4 * c + q) ^ l16);
        u32x4_t xh[4], xm[4], xlo[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t* r = xb + 16 * i * (kBf3QK / 2) + pos;
          xh[i] = *reinterpret_cast<const u32x4_t*>(r);
          xm[i] = *reinterpret_cast<const u32x4_t*>(r + kBf3Plane / 2);
          xlo[i] = *reinterpret_cast<const u32x4_t*>(r + kBf3Plane);
        }
        const int hn = h + kP < NQ * NC ? h + kP : NQ * NC - 1;  // clamped: the same loads every iteration
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          u32x4_t wh, wm, wlo;
          split_bf16x3(wb[p][j][0], wb[p][j][1], wh, wm, wlo);
#pragma unroll
          for (int i = 0; i < 4; ++i) {  // small terms first
            f32x4_t a = acc[i][j];
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xm[i]), as_bf16x8(wm), a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xlo[i]), as_bf16x8(wh), a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xh[i]), as_bf16x8(wlo), a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xm[i]), as_bf16x8(wh), a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xh[i]), as_bf16x8(wm), a, 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xh[i]), as_bf16x8(wh), a, 0, 0, 0);
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          wb[p][j][0] = ldw(wl + j * wj + 32 * hn);
          wb[p][j][1] = ldw(wl + j * wj + 32 * hn + 4);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the refill here (the scheduler would sink it to its use)
      }
    }
    if (qt + 1 < NQ) {
      __syncthreads();  // buffer qt & 1 fully read; the previous quarter's split writes visible
      if (qt + 2 < NQ) {
        store_quarter(qt & 1);  // quarter qt + 2
        if (qt + 3 < NQ) load_quarter(qt + 3);
      }
    }
  }
  if constexpr (kLN) {
    mlp_epilogue(acc, r0, K, w, w_ld, bias, e0, e1, e_ld, gamma, beta, eps, slope, y, y_ld, R, red, stat);
  } else {  // acc[i][j][e]: row 16 i + 4 q + e, column 64 wv + 16 j + l16
    float cb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) cb[j] = bias[64 * wv + 16 * j + l16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = r0 + 16 * i + 4 * q + e;
        if (row >= R) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) y[row * y_ld + 64 * wv + 16 * j + l16] = acc[i][j][e] + cb[j];
      }
  }
}

// decoder.py:106-117 — param = harmonic_proj(hidden), magnitudes = noise_proj(hidden) — as ONE launch on the
// bf16 matrix cores with the fp32-accurate three-term split (the six products of linear_bf3_kernel), reading
// both layers' parameters where they lie: output column c < n1 is W1 row c, n1 <= c < n1 + n2 is W2 row
// c - n1.  K = 512 (the decoder's hidden size).  A workgroup: 64 rows x 192 columns (blockIdx.y: the 192-column
// block); x is split once per workgroup into LDS planes a quarter of K at a time (linear_bf3_kernel's layout and
// pipeline).  The 8 waves are 4 column groups of 48 x 2 halves of K: wave (cg, kh) takes columns 48 cg .. + 47
// for ALL 64 rows (4 x 3 tiles, 72 MFMAs per 32-wide chunk) over the chunks of parity kh, splitting its own W
// rows from a register ring, so every W element is split once per workgroup; the kh = 1 half is added to the
// kh = 0 half through LDS at the end (the x planes' space), one fp32 add per output.  At config 2 (12,800 x 512
// -> 166) 200 workgroups, one per CU: 27.8 us against 32.1 us for 2 row halves x 4 column groups (each W
// element split twice, 36 MFMAs per split) and 34.5 us for round 5's stacking launch + hipBLASLt GEMM
// (profiles/r06y_projections_kernel.log).
constexpr int kProjCols = 192;  // output columns per workgroup
__global__ void __launch_bounds__(512) proj_bf3_sk_kernel(
    const float* __restrict__ x, int64_t x_ld, const float* __restrict__ w1, int64_t w1_ld,
    const float* __restrict__ b1, int n1, const float* __restrict__ w2, int64_t w2_ld, const float* __restrict__ b2,
    int n2, float* __restrict__ y, int64_t y_ld, int64_t R) {
  constexpr int K = 512, NQ = K / kBf3QK, NC = kBf3QK / 32, kP = 2, NH = NQ * NC;
  static_assert(NC == 2 * kP, "one ring slot per chunk parity step");
  __shared__ __attribute__((aligned(16))) uint32_t xs[2 * 3 * kBf3Plane / 2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int q = lane >> 4, l16 = lane & 15;
  const int kh = wv & 1, cg = wv >> 1;
  const int64_t r0 = (int64_t)blockIdx.x * kMlpRows;
  const int c0 = blockIdx.y * kProjCols + 48 * cg;
  const int n = n1 + n2;
  const float* wl[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = c0 + 16 * j + l16;
    wl[j] = (c < n1 ? w1 + (int64_t)c * w1_ld : c < n ? w2 + (int64_t)(c - n1) * w2_ld : w1) + 8 * q;
  }
  // this wave's chunks: h = 2 s + kh, s = 0 .. NH / 2 - 1; ring slot s % kP
  float4 wb[kP][3][2];
#pragma unroll
  for (int p = 0; p < kP; ++p)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      wb[p][j][0] = *reinterpret_cast<const float4*>(wl[j] + 32 * (2 * p + kh));
      wb[p][j][1] = *reinterpret_cast<const float4*>(wl[j] + 32 * (2 * p + kh) + 4);
    }
  const int srow = t >> 3, sq = 2 * (t & 7);
  const float* xsrc = x + (r0 + srow < R ? r0 + srow : R - 1) * x_ld + 8 * sq;  // rows >= R: never stored
  float4 xv[4];
  auto load_quarter = [&](int qt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) xv[i] = *reinterpret_cast<const float4*>(xsrc + kBf3QK * qt + 4 * i);
  };
  auto store_quarter = [&](int buf) {
    uint32_t* base = xs + buf * (3 * kBf3Plane / 2) + srow * (kBf3QK / 2);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      u32x4_t hq, mq, lq;
      split_bf16x3(xv[2 * e], xv[2 * e + 1], hq, mq, lq);
      const int pos = 4 * ((sq + e) ^ (srow & 15));  // uint32 offset of the quad
      *reinterpret_cast<u32x4_t*>(base + pos) = hq;
      *reinterpret_cast<u32x4_t*>(base + kBf3Plane / 2 + pos) = mq;
      *reinterpret_cast<u32x4_t*>(base + kBf3Plane + pos) = lq;
    }
  };
  load_quarter(0);
  store_quarter(0);
  load_quarter(1);
  store_quarter(1);
  load_quarter(2);  // in flight under quarter 0
  __syncthreads();
  f32x4_t acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  for (int qt = 0; qt < NQ; ++qt) {
    const uint32_t* xb = xs + (qt & 1) * (3 * kBf3Plane / 2) + l16 * (kBf3QK / 2);  // row 16 i + l16: row & 15 = l16
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      const int c = 2 * p + kh, h = qt * NC + c;
      const int pos = 4 * ((4 * c + q) ^ l16);
      u32x4_t xh[4], xm[4], xlo[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t* r = xb + 16 * i * (kBf3QK / 2) + pos;
        xh[i] = *reinterpret_cast<const u32x4_t*>(r);
        xm[i] = *reinterpret_cast<const u32x4_t*>(r + kBf3Plane / 2);
        xlo[i] = *reinterpret_cast<const u32x4_t*>(r + kBf3Plane);
      }
      const int hn = h + 2 * kP < NH ? h + 2 * kP : NH - 2 + kh;  // clamped: the same loads every iteration
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        u32x4_t wh, wm, wlo;
        split_bf16x3(wb[p][j][0], wb[p][j][1], wh, wm, wlo);
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // small terms first
          f32x4_t a = acc[i][j];
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xm[i]), as_bf16x8(wm), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xlo[i]), as_bf16x8(wh), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xh[i]), as_bf16x8(wlo), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xm[i]), as_bf16x8(wh), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xh[i]), as_bf16x8(wm), a, 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(xh[i]), as_bf16x8(wh), a, 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        wb[p][j][0] = *reinterpret_cast<const float4*>(wl[j] + 32 * hn);
        wb[p][j][1] = *reinterpret_cast<const float4*>(wl[j] + 32 * hn + 4);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the refill here (the scheduler would sink it to its use)
    }
    if (qt + 1 < NQ) {
      __syncthreads();  // buffer qt & 1 fully read; the previous quarter's split writes visible
      if (qt + 2 < NQ) {
        store_quarter(qt & 1);  // quarter qt + 2
        if (qt + 3 < NQ) load_quarter(qt + 3);
      }
    }
  }
  // the kh = 1 half through LDS ([cg][48 values][64 lanes] floats in the x planes' space)
  __syncthreads();
  float* red = reinterpret_cast<float*>(xs) + cg * 48 * 64 + lane;
  if (kh == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[((3 * i + j) * 4 + e) * 64] = acc[i][j][e];
  }
  __syncthreads();
  if (kh == 1) return;
  // acc[i][j][e]: row 16 i + 4 q + e, column c0 + 16 j + l16
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = c0 + 16 * j + l16;
    if (c >= n) continue;
    const float cb = c < n1 ? b1[c] : b2[c - n1];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = r0 + 16 * i + 4 * q + e;
        if (row < R) y[row * y_ld + c] = (acc[i][j][e] + red[((3 * i + j) * 4 + e) * 64]) + cb;
      }
  }
}

// Weight gradient of a Linear under autograd (training: the decoder MLPs' Linears, the GRU's W_ih / W_hh):
// dW[m][n] = sum_r dY[r][m] X[r][n] — a product over the ROW index of two row-major matrices, on the bf16 matrix
// cores with the exact three-term split (six products, fp32-accurate).  A workgroup: a 64 (m) x 128 (n) tile of dW
// over one of S row ranges (split-K; the S per-tile partials are summed in range order by wgrad_sum_kernel, so the
// result does not depend on scheduling).  Per 32-row chunk each thread loads 8 consecutive rows of one column
// (coalesced across the wave's lanes), splits them and writes the 16-byte [column][8 rows] quads of the three
// planes into LDS — the MFMA fragments' k-major layout, quads swizzled per column so that a fragment read is
// conflict-free — double-buffered with one barrier per chunk; the loads run two chunks ahead (two register sets)
// under the current chunk's 48 MFMAs per wave (wave w: m-tile w x the 8 n-tiles).  Row ranges are sliced by XCD
// (S a multiple of 8, workgroup b on XCD b % 8 takes ranges of slice b % 8): an XCD streams only its eighth of
// dY and X from HBM and serves the tiles' re-reads from its own L2.
constexpr int kWgN = 128, kWgR = 32, kWgBufs = 1;
// LDS quad of [column][row group q]: the group index XOR-swizzled by column bits 1..3 so that both the fragment
// reads (16-lane groups of 16 columns x 4 row groups) and the 16-byte stores (8-lane groups of 8 columns) are
// conflict-free
__device__ __forceinline__ int wgrad_quad(int col, int q) {
  return col * (kWgR / 8) + (q ^ ((0x78 >> (2 * ((col >> 2) & 3))) & 3) ^ ((col >> 1) & 1));
}
// split_bf16x3 with the two exact residual subtractions on packed fp32 (v_pk_add_f32): the same bits
typedef float f32x2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void wgrad_split(const float* v, u32x4_t& hi, u32x4_t& mid, u32x4_t& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t u0 = __float_as_uint(v[2 * e]), u1 = __float_as_uint(v[2 * e + 1]);
    const f32x2v_t x = {v[2 * e], v[2 * e + 1]};
    const f32x2v_t h = {__uint_as_float(u0 & 0xffff0000u), __uint_as_float(u1 & 0xffff0000u)};
    const f32x2v_t r = x - h;  // exact
    const uint32_t m0 = __float_as_uint(r.x) & 0xffff0000u, m1 = __float_as_uint(r.y) & 0xffff0000u;
    const f32x2v_t l = r - (f32x2v_t){__uint_as_float(m0), __uint_as_float(m1)};  // exact
    hi[e] = __builtin_amdgcn_perm(u1, u0, 0x07060302u);
    mid[e] = __builtin_amdgcn_perm(m1, m0, 0x07060302u);
    lo[e] = __builtin_amdgcn_perm(__float_as_uint(l.y), __float_as_uint(l.x), 0x07060302u);
  }
}
template <int WM>  // m-tiles per wave: the workgroup's dW tile is 64 WM x 128
__global__ void __launch_bounds__(256) wgrad_bf3_kernel(const float* __restrict__ dy, int64_t dy_ld,
                                                        const float* __restrict__ x, int64_t x_ld,
                                                        float* __restrict__ part, int64_t R, int M, int N, int S,
                                                        int64_t rows_per_split, int Mr, int Nr) {
  // M, N: the partials' padded extents (multiples of the tile); Mr, Nr: dW's own (columns of dY and X)
  constexpr int TM = 64 * WM;
  // [buffer][plane][column][32 rows] bf16: A (dY) TM columns, B (X) 128 columns
  __shared__ __attribute__((aligned(16))) uint32_t la[kWgBufs][3][TM * kWgR / 2];
  __shared__ __attribute__((aligned(16))) uint32_t lb[kWgBufs][3][kWgN * kWgR / 2];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int q = lane >> 4, l16 = lane & 15;
  // workgroup -> (split, tile): XCD b % 8 owns splits [(b % 8) S/8, (b % 8 + 1) S/8)
  const int b = blockIdx.x, per_xcd = S >> 3, i = b >> 3;
  const int split = (b & 7) * per_xcd + i % per_xcd, tile = i / per_xcd, mt = M / TM;
  const int m0 = (tile % mt) * TM, n0 = (tile / mt) * kWgN;
  const int64_t rb = (int64_t)split * rows_per_split;
  const int64_t re = min(rb + rows_per_split, R);
  const int nch = re > rb ? (int)((re - rb + kWgR - 1) / kWgR) : 0;
  // load tasks: A column t % TM, row groups t / TM + (4 / WM) h (h < WM); B column t & 127, row groups t >> 7 and
  // + 2.  Raw buffer loads over the range's rows: the row offset is a wave-uniform SGPR operand, the lane's column
  // offset a constant VGPR, and rows at or past the range's end lie outside the descriptor's records and read 0.
  const int am = t & (TM - 1), bn = t & 127;
  const int ag = __builtin_amdgcn_readfirstlane(t / TM), bg = __builtin_amdgcn_readfirstlane(t >> 7);
  const int rows_here = re > rb ? (int)(re - rb) : 0;
  const int a_ld4 = (int)(dy_ld * 4), b_ld4 = (int)(x_ld * 4);
  // records end at the range's last element: columns past dW's edge read the next row (their products land in
  // the padding of the partials) or, on the last row, zero — never memory past the operands
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(dy + rb * dy_ld), (short)0, rows_here ? (rows_here - 1) * a_ld4 + 4 * Mr : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rbx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x + rb * x_ld), (short)0, rows_here ? (rows_here - 1) * b_ld4 + 4 * Nr : 0, 0x00020000);
  const int va_off = (m0 + am) * 4, vb_off = (n0 + bn) * 4;
  struct Regs {
    float a[WM][8], b[2][8];
  };
  auto load = [&](int c, Regs& v) {
    const int ra0 = (c * kWgR + 8 * ag) * a_ld4;
    const int rb0 = (c * kWgR + 8 * bg) * b_ld4;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int h = 0; h < WM; ++h)
        v.a[h][k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, va_off, ra0 + (32 / WM * h + k) * a_ld4, 0));
#pragma unroll
      for (int h = 0; h < 2; ++h)
        v.b[h][k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rbx, vb_off, rb0 + (16 * h + k) * b_ld4, 0));
    }
  };
  auto store = [&](int buf, const Regs& v) {
    u32x4_t hi, mi, lo;
#pragma unroll
    for (int h = 0; h < WM; ++h) {
      wgrad_split(v.a[h], hi, mi, lo);
      const int qa = wgrad_quad(am, ag + 4 / WM * h);
      reinterpret_cast<u32x4_t*>(la[buf][0])[qa] = hi;
      reinterpret_cast<u32x4_t*>(la[buf][1])[qa] = mi;
      reinterpret_cast<u32x4_t*>(la[buf][2])[qa] = lo;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      wgrad_split(v.b[h], hi, mi, lo);
      const int qb = wgrad_quad(bn, bg + 2 * h);
      reinterpret_cast<u32x4_t*>(lb[buf][0])[qb] = hi;
      reinterpret_cast<u32x4_t*>(lb[buf][1])[qb] = mi;
      reinterpret_cast<u32x4_t*>(lb[buf][2])[qb] = lo;
    }
  };
  f32x4_t acc[WM][8];
#pragma unroll
  for (int u = 0; u < WM; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[u][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int buf) {
    // A fragment of m-tile u: row (m) 16 (WM w + u) + l16, k = 8 q .. + 7; B fragment of n-tile j: column 16 j + l16
    u32x4_t ah[WM], am_[WM], al[WM];
#pragma unroll
    for (int u = 0; u < WM; ++u) {
      const int qa = wgrad_quad(16 * (WM * w + u) + l16, q);
      ah[u] = reinterpret_cast<const u32x4_t*>(la[buf][0])[qa];
      am_[u] = reinterpret_cast<const u32x4_t*>(la[buf][1])[qa];
      al[u] = reinterpret_cast<const u32x4_t*>(la[buf][2])[qa];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int qb = wgrad_quad(16 * j + l16, q);
      const u32x4_t bh = reinterpret_cast<const u32x4_t*>(lb[buf][0])[qb];
      const u32x4_t bm = reinterpret_cast<const u32x4_t*>(lb[buf][1])[qb];
      const u32x4_t bl = reinterpret_cast<const u32x4_t*>(lb[buf][2])[qb];
#pragma unroll
      for (int u = 0; u < WM; ++u) {
        f32x4_t a = acc[u][j];  // small terms first
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(am_[u]), as_bf16x8(bm), a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(al[u]), as_bf16x8(bh), a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(ah[u]), as_bf16x8(bl), a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(am_[u]), as_bf16x8(bh), a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(ah[u]), as_bf16x8(bm), a, 0, 0, 0);
        acc[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(ah[u]), as_bf16x8(bh), a, 0, 0, 0);
      }
    }
  };
  // chunk k's loads land in register set k & 1; iteration c: MFMAs on the LDS tile, chunk c + 1 into LDS behind a
  // barrier, then chunk c + 3's loads into the set chunk c + 1 has left
  Regs r0, r1;
  if (nch > 0) {
    load(0, r0);
    store(0, r0);
    if (nch > 1) load(1, r1);
    if (nch > 2) load(2, r0);
  }
  __syncthreads();
  auto step = [&](int c, Regs& nxt) {
    mma(c & (kWgBufs - 1));
    if (kWgBufs == 1) __syncthreads();
    if (c + 1 < nch) store((c + 1) & (kWgBufs - 1), nxt);
    if (c + 3 < nch) load(c + 3, nxt);
    __syncthreads();
  };
  for (int c = 0; c < nch; c += 2) {
    step(c, r1);
    if (c + 1 < nch) step(c + 1, r0);
  }
  // acc[u][j][e]: m = m0 + 16 (WM w + u) + 4 q + e, n = n0 + 16 j + l16
  float* pp = part + (int64_t)split * M * N;
#pragma unroll
  for (int u = 0; u < WM; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        pp[(int64_t)(m0 + 16 * (WM * w + u) + 4 * q + e) * N + n0 + 16 * j + l16] = acc[u][j][e];
}

// dW = the S partials ([S][M][N] padded) summed in range order, written with row stride dw_ld: 4 columns per
// thread, one 16-byte store where dW's row holds all four and is aligned, else element stores
__global__ void __launch_bounds__(256) wgrad_sum_kernel(const float* __restrict__ part, int S, int M, int N, int Mr,
                                                        int Nr, float* __restrict__ dw, int64_t dw_ld, int vec) {
  const int64_t i4 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i4 >= (int64_t)Mr * N / 4) return;
  const int64_t m = (4 * i4) / N, n = 4 * i4 - m * N;
  if (n >= Nr) return;
  float4 a = reinterpret_cast<const float4*>(part)[i4];
  for (int s = 1; s < S; ++s) {
    const float4 b = reinterpret_cast<const float4*>(part + (int64_t)s * M * N)[i4];
    a = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
  float* o = dw + m * dw_ld + n;
  if (vec && n + 4 <= Nr) {
    *reinterpret_cast<float4*>(o) = a;
  } else {
    const float v[4] = {a.x, a.y, a.z, a.w};
    for (int e = 0; e < 4 && n + e < Nr; ++e) o[e] = v[e];
  }
}

static int wgrad_splits_for(int64_t tiles) {
  // a multiple of 8 (one slice of row ranges per XCD) giving >= 512 workgroups (more ranges cost more partial
  // traffic than the extra occupancy returns: 512 x 512 at 1024 workgroups measured 70 us, at 512 61 us)
  const int64_t k = std::max<int64_t>(1, (64 + tiles - 1) / tiles);
  return (int)std::min<int64_t>(8 * k, 64);
}
// m-tiles per wave: 128-row dW tiles (twice the MFMAs per split element, 2 waves per SIMD) where they divide M and
// fill whole 512-workgroup rounds, else 64-row tiles (4 waves per SIMD).  Same box, us (profiles/r06w_weight_grad.log):
// 512 x 512 60 vs 64, W_ih 1536 x 1024 288 vs 270 (768 workgroups = 1.5 rounds), W_hh 1536 x 512 131 vs 129.
static int wgrad_wm(int M, int N) {
  if (M % 128) return 1;
  const int64_t tiles = (int64_t)(M / 128) * ((N + kWgN - 1) / kWgN);
  return (tiles * wgrad_splits_for(tiles)) % 512 == 0 ? 2 : 1;
}
struct WgradShape {
  int wm, S, Mp, Np;  // tile height / 64, row ranges, padded extents of the partials
};
static WgradShape wgrad_shape(int M, int N) {
  WgradShape g;
  g.wm = wgrad_wm(M, N);
  g.Mp = (M + 64 * g.wm - 1) / (64 * g.wm) * (64 * g.wm);
  g.Np = (N + kWgN - 1) / kWgN * kWgN;
  g.S = wgrad_splits_for((int64_t)(g.Mp / (64 * g.wm)) * (g.Np / kWgN));
  return g;
}

// The two projections' parameters stacked into one zero-padded [n_pad, K] weight and [n_pad] bias (a
// caller buffer): the GEMM that follows runs at a padded width hipBLASLt is fast at (28-30 us for 192
// outputs against 38-39 us for the 166 of decoder.py:87-88 at config 2).  One launch, fresh every call.
__global__ void __launch_bounds__(256) stack_rows_kernel(const float* __restrict__ w1, int64_t w1_ld, const float* __restrict__ b1,
                                                         int n1, const float* __restrict__ w2, int64_t w2_ld,
                                                         const float* __restrict__ b2, int n2, int K,
                                                         float* __restrict__ w, float* __restrict__ b, int n_pad) {
  const int r = blockIdx.x;
  const float* src = r < n1 ? w1 + (int64_t)r * w1_ld : r < n1 + n2 ? w2 + (int64_t)(r - n1) * w2_ld : nullptr;
  for (int k = threadIdx.x; k < K; k += 256) w[(int64_t)r * K + k] = src ? src[k] : 0.0f;
  if (threadIdx.x == 0) b[r] = r < n1 ? b1[r] : r < n1 + n2 ? b2[r - n1] : 0.0f;
}

}  // namespace
}  // namespace ddsp

using namespace ddsp;

extern "C" {

int ddsp_hip_dense_rows(const ddsp_hip_dense_problem* problems, int n_problems, int64_t rows, void* stream) {
  if (!problems || n_problems < 1 || n_problems > DDSP_HIP_DENSE_MAX_PROBLEMS || rows < 0) return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  if (rows > kMaxRows) return DDSP_HIP_ERANGE;
  DenseArgs args{};
  args.rows = (int)rows;
  int64_t max_n = 0, max_k = 0;
  for (int i = 0; i < n_problems; ++i) {
    const ddsp_hip_dense_problem& P = problems[i];
    if (!P.weight || !P.y || P.out_features < 1 || P.n_inputs < 1 || P.n_inputs > DDSP_HIP_DENSE_MAX_INPUTS ||
        P.ldy < P.out_features)
      return DDSP_HIP_EINVAL;
    int64_t K = 0;
    for (int s = 0; s < P.n_inputs; ++s) {
      const ddsp_hip_dense_input& in = P.inputs[s];
      if (!in.x || in.width < 1 || (in.gamma && !in.beta) || (in.w1 && !in.b1)) return DDSP_HIP_EINVAL;
      if (!in.w1 && in.ld < in.width) return DDSP_HIP_EINVAL;
      if (in.width > 64 * kKL) return DDSP_HIP_ERANGE;
      K += in.width;
    }
    max_n = std::max<int64_t>(max_n, P.out_features);
    max_k = std::max(max_k, K);
    args.p[i] = P;
  }
  const size_t shm = sizeof(float) * (size_t)rows * (size_t)max_k;
  if (max_k > 64 * kKL || max_n > (int64_t)65535 * kOutPerWG) return DDSP_HIP_ERANGE;
  const dim3 grid((unsigned)((max_n + kOutPerWG - 1) / kOutPerWG), (unsigned)n_problems);
  hipLaunchKernelGGL(dense_rows_kernel, grid, dim3(kDenseNT), shm, reinterpret_cast<hipStream_t>(stream), args);
  return launch_status();
}

int ddsp_hip_layer_norm_leaky_relu(const float* x, int64_t x_ld, const float* w1, const float* b1, const float* gamma,
                                   const float* beta, float eps, float slope, float* y, int64_t y_ld, int64_t rows,
                                   int64_t cols, void* stream) {
  if (rows < 0 || cols < 1 || !gamma || !beta || (!w1) != (!b1)) return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  if (!x || !y || y_ld < cols || (!w1 && x_ld < cols) || (w1 && x_ld < 1)) return DDSP_HIP_EINVAL;
  const uintptr_t al = reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(gamma) |
                       reinterpret_cast<uintptr_t>(beta) | (w1 ? reinterpret_cast<uintptr_t>(w1) |
                       reinterpret_cast<uintptr_t>(b1) : reinterpret_cast<uintptr_t>(x));
  if ((cols != 512 && cols != 1024) || (al & 15) || (y_ld & 3) || (!w1 && (x_ld & 3)) || rows > (int64_t)4 * 0x7fffffff)
    return DDSP_HIP_ERANGE;  // callers keep torch's LayerNorm + LeakyReLU
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (cols == 512)
    hipLaunchKernelGGL(ln_leaky_kernel<2>, grid, dim3(256), 0, st, x, x_ld, w1, b1, gamma, beta, eps, slope, y, y_ld, rows);
  else
    hipLaunchKernelGGL(ln_leaky_kernel<4>, grid, dim3(256), 0, st, x, x_ld, w1, b1, gamma, beta, eps, slope, y, y_ld, rows);
  return launch_status();
}

size_t ddsp_hip_layer_norm_leaky_relu_backward_workspace_size(int64_t cols) {
  return cols > 0 ? sizeof(float) * (size_t)kLnBwdGrid * 2 * (size_t)cols : 0;
}

int ddsp_hip_layer_norm_leaky_relu_backward(const float* x, int64_t x_ld, const float* gamma, const float* beta, float eps,
                                            float slope, const float* grad_y, int64_t dy_ld, float* grad_x, int64_t dx_ld,
                                            float* grad_gamma, float* grad_beta, int64_t rows, int64_t cols, void* ws,
                                            size_t ws_bytes, void* stream) {
  if (rows < 0 || cols < 1 || !gamma || !beta) return DDSP_HIP_EINVAL;
  if (rows == 0) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (grad_gamma && hipMemsetAsync(grad_gamma, 0, sizeof(float) * (size_t)cols, st) != hipSuccess) return DDSP_HIP_ELAUNCH;
    if (grad_beta && hipMemsetAsync(grad_beta, 0, sizeof(float) * (size_t)cols, st) != hipSuccess) return DDSP_HIP_ELAUNCH;
    return DDSP_HIP_OK;
  }
  if (!x || !grad_y || !grad_x || x_ld < cols || dy_ld < cols || dx_ld < cols) return DDSP_HIP_EINVAL;
  const bool params = grad_gamma || grad_beta;
  if (params && (!ws || ws_bytes < ddsp_hip_layer_norm_leaky_relu_backward_workspace_size(cols))) return DDSP_HIP_EWORKSPACE;
  const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(grad_y) |
                       reinterpret_cast<uintptr_t>(grad_x) | reinterpret_cast<uintptr_t>(gamma) |
                       reinterpret_cast<uintptr_t>(beta);
  if ((cols != 512 && cols != 1024) || (al & 15) || (x_ld & 3) || (dy_ld & 3) || (dx_ld & 3))
    return DDSP_HIP_ERANGE;  // callers keep torch's LayerNorm + LeakyReLU backward
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* part = params ? reinterpret_cast<float*>(ws) : nullptr;
  const int64_t need = (rows + 3) / 4;
  const unsigned grid = (unsigned)std::min<int64_t>(kLnBwdGrid, need);
  if (cols == 512)
    hipLaunchKernelGGL(ln_leaky_bwd_kernel<2>, dim3(grid), dim3(256), 0, st, x, x_ld, gamma, beta, eps, slope, grad_y,
                       dy_ld, grad_x, dx_ld, part, rows);
  else
    hipLaunchKernelGGL(ln_leaky_bwd_kernel<4>, dim3(grid), dim3(256), 0, st, x, x_ld, gamma, beta, eps, slope, grad_y,
                       dy_ld, grad_x, dx_ld, part, rows);
  if (params)
    hipLaunchKernelGGL(ln_leaky_bwd_sum_kernel, dim3((unsigned)((2 * cols + 63) / 64)), dim3(256), 0, st, part,
                       (int)grid, (int)cols, grad_gamma, grad_beta);
  return launch_status();
}

int ddsp_hip_mlp_block(const float* x, int64_t x_ld, int64_t in_features, const float* w, int64_t w_ld,
                       const float* bias, const float* e0, const float* e1, int64_t e_ld, const float* gamma,
                       const float* beta, float eps, float slope, float* y, int64_t y_ld, int64_t rows,
                       int64_t out_features, int flags, void* stream) {
  if (rows < 0 || in_features < 1 || !w || !bias || !gamma || !beta || (!e0 && e1)) return DDSP_HIP_EINVAL;
  if (flags & ~DDSP_HIP_MLP_EXACT_F32) return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  const int64_t extra = e1 ? 2 : e0 ? 1 : 0;
  if (!x || !y || x_ld < in_features || w_ld < in_features + extra || y_ld < out_features || (extra && e_ld < 1))
    return DDSP_HIP_EINVAL;
  if (out_features != kMlpN || in_features > INT32_MAX || (rows + kMlpRows - 1) / kMlpRows > INT32_MAX)
    return DDSP_HIP_ERANGE;  // callers keep the GEMM + layer_norm_leaky_relu route
  const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w);
  const int vec = in_features % 4 ? 1 : (x_ld % 4 == 0 && w_ld % 4 == 0 && (al & 15) == 0) ? 4
                                      : (x_ld % 2 == 0 && w_ld % 2 == 0 && (al & 7) == 0) ? 2 : 1;
  const dim3 grid((unsigned)((rows + kMlpRows - 1) / kMlpRows));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool x16 = x_ld % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (in_features == kMlpResK && x16 && (flags & DDSP_HIP_MLP_EXACT_F32) == 0 && vec == 4)  // the decoder's blocks
    hipLaunchKernelGGL((linear_bf3_kernel<2, kMlpResK, true>), grid, dim3(512), 0, st, x, x_ld, w, w_ld, bias, e0, e1,
                       e_ld, gamma, beta, eps, slope, y, y_ld, rows);
  else if (in_features == kMlpResK && x16 && (flags & DDSP_HIP_MLP_EXACT_F32) == 0 && w_ld % 2 == 0 &&
           (reinterpret_cast<uintptr_t>(w) & 7) == 0)  // W rows 8-byte aligned: the out_mlp's first block
    hipLaunchKernelGGL((linear_bf3_kernel<2, kMlpResK, true, true>), grid, dim3(512), 0, st, x, x_ld, w, w_ld, bias, e0,
                       e1, e_ld, gamma, beta, eps, slope, y, y_ld, rows);
  else if (in_features == kMlpResK && vec == 4)  // x resident, W streamed to registers, f32 MFMA
    hipLaunchKernelGGL(mlp_block_res_kernel<4>, grid, dim3(512), 0, st, x, x_ld, w, w_ld, bias, e0, e1, e_ld, gamma,
                       beta, eps, slope, y, y_ld, rows);
  else if (vec == 4)
    hipLaunchKernelGGL(mlp_block_kernel<4>, grid, dim3(512), 0, st, x, x_ld, (int)in_features, w, w_ld, bias, e0, e1,
                       e_ld, gamma, beta, eps, slope, y, y_ld, rows);
  else if (vec == 2)
    hipLaunchKernelGGL(mlp_block_kernel<2>, grid, dim3(512), 0, st, x, x_ld, (int)in_features, w, w_ld, bias, e0, e1,
                       e_ld, gamma, beta, eps, slope, y, y_ld, rows);
  else
    hipLaunchKernelGGL(mlp_block_kernel<1>, grid, dim3(512), 0, st, x, x_ld, (int)in_features, w, w_ld, bias, e0, e1,
                       e_ld, gamma, beta, eps, slope, y, y_ld, rows);
  return launch_status();
}

int ddsp_hip_linear(const float* x, int64_t x_ld, int64_t in_features, const float* w, int64_t w_ld,
                    const float* bias, float* y, int64_t y_ld, int64_t rows, int64_t out_features, void* stream) {
  if (rows < 0 || in_features < 1 || out_features < 1 || !w || !bias) return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  if (!x || !y || x_ld < in_features || w_ld < in_features || y_ld < out_features) return DDSP_HIP_EINVAL;
  const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w);
  if ((in_features != 512 && in_features != 1024 && in_features != 1536) || out_features % kMlpN || (al & 15) ||
      (x_ld & 3) || (w_ld & 3) ||
      (rows + kMlpRows - 1) / kMlpRows > INT32_MAX || out_features / kMlpN > 65535)
    return DDSP_HIP_ERANGE;  // callers keep their library GEMM
  const dim3 grid((unsigned)((rows + kMlpRows - 1) / kMlpRows), (unsigned)(out_features / kMlpN));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (in_features == 1536)  // the GRU input gradient (3 gates x 512 -> 1024 under autograd)
    hipLaunchKernelGGL((linear_bf3_kernel<2, 1536, false>), grid, dim3(512), 0, st, x, x_ld, w, w_ld, bias, nullptr,
                       nullptr, 0, nullptr, nullptr, 0.0f, 0.0f, y, y_ld, rows);
  else if (in_features == 1024)
    hipLaunchKernelGGL((linear_bf3_kernel<2, 1024, false>), grid, dim3(512), 0, st, x, x_ld, w, w_ld, bias, nullptr,
                       nullptr, 0, nullptr, nullptr, 0.0f, 0.0f, y, y_ld, rows);
  else
    hipLaunchKernelGGL((linear_bf3_kernel<2, 512, false>), grid, dim3(512), 0, st, x, x_ld, w, w_ld, bias, nullptr,
                       nullptr, 0, nullptr, nullptr, 0.0f, 0.0f, y, y_ld, rows);
  return launch_status();
}

int ddsp_hip_projections(const float* x, int64_t x_ld, int64_t in_features, const float* w1, int64_t w1_ld,
                         const float* b1, int64_t n1, const float* w2, int64_t w2_ld, const float* b2, int64_t n2,
                         float* y, int64_t y_ld, int64_t rows, void* stream) {
  if (rows < 0 || in_features < 1 || n1 < 1 || n2 < 0 || !w1 || !b1 || (n2 > 0 && (!w2 || !b2))) return DDSP_HIP_EINVAL;
  if (rows == 0) return DDSP_HIP_OK;
  if (!x || !y || x_ld < in_features || w1_ld < in_features || (n2 > 0 && w2_ld < in_features) || y_ld < n1 + n2)
    return DDSP_HIP_EINVAL;
  if (n2 == 0) {  // one layer: the second pointer set is never read
    w2 = w1;
    w2_ld = w1_ld;
    b2 = b1;
  }
  const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w1) | reinterpret_cast<uintptr_t>(w2);
  if (in_features != 512 || (al & 15) || (x_ld & 3) || (w1_ld & 3) || (w2_ld & 3) || n1 + n2 > 65535 * kProjCols ||
      (rows + kMlpRows - 1) / kMlpRows > INT32_MAX)
    return DDSP_HIP_ERANGE;  // callers keep their library GEMM
  const dim3 grid((unsigned)((rows + kMlpRows - 1) / kMlpRows), (unsigned)((n1 + n2 + kProjCols - 1) / kProjCols));
  hipLaunchKernelGGL(proj_bf3_sk_kernel, grid, dim3(512), 0, reinterpret_cast<hipStream_t>(stream), x, x_ld, w1, w1_ld, b1,
                     (int)n1, w2, w2_ld, b2, (int)n2, y, y_ld, rows);
  return launch_status();
}

size_t ddsp_hip_linear_weight_grad_workspace_size(int64_t rows, int64_t out_features, int64_t in_features) {
  if (rows < 1 || out_features < 1 || in_features < 1 || out_features > (1 << 24) || in_features > (1 << 24)) return 0;
  const WgradShape g = wgrad_shape((int)out_features, (int)in_features);
  return sizeof(float) * (size_t)g.S * (size_t)g.Mp * (size_t)g.Np;
}

int ddsp_hip_linear_weight_grad(const float* grad_y, int64_t dy_ld, const float* x, int64_t x_ld, float* grad_w,
                                int64_t dw_ld, int64_t rows, int64_t out_features, int64_t in_features, void* ws,
                                size_t ws_bytes, void* stream) {
  if (rows < 0 || out_features < 1 || in_features < 1) return DDSP_HIP_EINVAL;
  if (!grad_w || dw_ld < in_features) return DDSP_HIP_EINVAL;
  if (rows > 0 && (!grad_y || !x || dy_ld < out_features || x_ld < in_features)) return DDSP_HIP_EINVAL;
  if (out_features > (1 << 24) || in_features > (1 << 24)) return DDSP_HIP_ERANGE;  // callers keep their library GEMM
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {
    for (int64_t m = 0; m < out_features; ++m)
      if (hipMemsetAsync(grad_w + m * dw_ld, 0, sizeof(float) * (size_t)in_features, st) != hipSuccess)
        return DDSP_HIP_ELAUNCH;
    return DDSP_HIP_OK;
  }
  const int M = (int)out_features, N = (int)in_features;
  const WgradShape g = wgrad_shape(M, N);
  const int64_t chunks = (rows + kWgR - 1) / kWgR;
  const int64_t per = ((chunks + g.S - 1) / g.S) * kWgR;  // rows per range (whole chunks; trailing ranges may be empty)
  const int64_t tiles = (int64_t)(g.Mp / (64 * g.wm)) * (g.Np / kWgN);
  // the grid, and 32-bit buffer offsets over one range (+ one chunk of rows past its end)
  if (tiles * g.S > INT32_MAX || (per + kWgR) * std::max(dy_ld, x_ld) * 4 > INT32_MAX) return DDSP_HIP_ERANGE;
  if (!ws || ws_bytes < ddsp_hip_linear_weight_grad_workspace_size(rows, out_features, in_features))
    return DDSP_HIP_EWORKSPACE;
  float* part = reinterpret_cast<float*>(ws);
  if (g.wm == 2)
    hipLaunchKernelGGL(wgrad_bf3_kernel<2>, dim3((unsigned)(tiles * g.S)), dim3(256), 0, st, grad_y, dy_ld, x, x_ld,
                       part, rows, g.Mp, g.Np, g.S, per, M, N);
  else
    hipLaunchKernelGGL(wgrad_bf3_kernel<1>, dim3((unsigned)(tiles * g.S)), dim3(256), 0, st, grad_y, dy_ld, x, x_ld,
                       part, rows, g.Mp, g.Np, g.S, per, M, N);
  const int vec = !(dw_ld & 3) && !(reinterpret_cast<uintptr_t>(grad_w) & 15);
  hipLaunchKernelGGL(wgrad_sum_kernel, dim3((unsigned)(((int64_t)M * g.Np / 4 + 255) / 256)), dim3(256), 0, st, part,
                     g.S, g.Mp, g.Np, M, N, grad_w, dw_ld, vec);
  return launch_status();
}

int ddsp_hip_stack_rows(const float* w1, int64_t w1_ld, const float* b1, int64_t n1, const float* w2, int64_t w2_ld,
                        const float* b2, int64_t n2, int64_t in_features, float* w, float* b, int64_t n_pad,
                        void* stream) {
  if (n1 < 1 || n2 < 0 || in_features < 1 || n_pad < n1 + n2 || !w1 || !b1 || !w || !b ||
      (n2 > 0 && (!w2 || !b2)) || w1_ld < in_features || (n2 > 0 && w2_ld < in_features))
    return DDSP_HIP_EINVAL;
  if (n_pad > INT32_MAX || in_features > INT32_MAX) return DDSP_HIP_ERANGE;
  hipLaunchKernelGGL(stack_rows_kernel, dim3((unsigned)n_pad), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), w1,
                     w1_ld, b1, (int)n1, w2, w2_ld, b2, (int)n2, (int)in_features, w, b, (int)n_pad);
  return launch_status();
}

}  // extern "C"
