// The decoder's recurrent layer on gfx950 (the network before the path;
// decoder.py:33-68 GRUDecoder, torch.nn.GRU(2*hidden, hidden, batch_first=True)).
//
// torch.nn.GRU, gate order (r, z, n):
//   r = sigmoid(xp_r + W_hr h + b_hr),  z = sigmoid(xp_z + W_hz h + b_hz),
//   n = tanh(xp_n + r * (W_hn h + b_hn)),  h' = (1 - z) * n + z * h
// where xp = x W_ih^T + b_ih for every time step at once is one plain GEMM (the caller's
// hipBLASLt matmul).  The recurrence is what MIOpen spends ~45 us per step on at batch 64,
// hidden 512: here one launch per step, 512 workgroups (hidden slices of 4 units x batch tiles
// of 16), each holding its 12 rows of W_hh in LDS and its batch tile's h chunk in registers; a
// step is a chain of latencies (load h and W, reduce, gate), so all of a step's loads are in flight
// together;
// the kernel boundary is the step's grid-wide barrier (no persistent spin, no residency
// requirement).  h_t is written straight into the output sequence, which is the next step's h.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"

namespace ddsp {
namespace {

constexpr int kHS = 4;    // hidden units per workgroup
// Tile shape (template arguments of both step kernels): kBS batch rows per workgroup x kKC k-chunks
// (threads per batch row), kBS * kKC = 512 threads.  (16, 32) where hidden % 128 == 0 — 7.7-7.9 us per
// step at config 2 against 8.4-8.5 for (32, 16) and 11.9 for (64, 8), profiles/r04i_gru_tiles.log —
// else (32, 16) (hidden % 64 == 0).

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// grid (H / kHS, ceil(B / kBS)); LDS: W slice [3 kHS][H] + per-wave partials [kNT / 64][3 kHS][kBS].
// A step is a chain of dependent latencies, not work (100 MFLOP per step at config 2), so every
// global load is issued before the first wait: the epilogue operands, this thread's h chunk and its
// share of the W slice (unpredicated, at clamped addresses; out-of-range values are never used),
// then one wait, the W slice to LDS, one barrier.  The k-chunk partials are summed inside each wave
// by lane exchanges first, so the epilogue wave reads kNT / 64 partials per gate instead of kKC.
// kH: the hidden size as a compile-time constant (512, the decoder's) so that the loads carry no
// predicates the compiler could turn into per-load branches and waits; 0 = any hidden size.
template <int kBS, int kKC, int kH>
__global__ void __launch_bounds__(kBS * kKC) gru_step_kernel(const float* __restrict__ xp, const float* __restrict__ w_hh,
                                                       const float* __restrict__ b_hh, const float* __restrict__ h_prev,
                                                       int64_t hp_ld, float* __restrict__ h_out, int64_t ho_ld,
                                                       int B, int H_arg, int64_t xp_ld, float* __restrict__ save,
                                                       int64_t save_plane, float* __restrict__ h_copy) {
  extern __shared__ float smem[];
  constexpr int kNT = kBS * kKC;
  constexpr int R = 3 * kHS;
  constexpr int kWaves = kNT / 64, kG = 64 / kBS;  // waves; k-chunk groups per wave
  static_assert(kBS <= 64 && 64 % kBS == 0 && kNT % 64 == 0, "tile shape");
  constexpr int kWV = 4;              // W slice float4s per thread per staging round
  const int H = kH ? kH : H_arg;
  float* W = smem;                    // [R][H]
  float* part = smem + R * H;         // [kWaves][R][kBS]
  const int j0 = blockIdx.x * kHS, b0 = blockIdx.y * kBS;
  const int tid = threadIdx.x;
  const int bl = tid % kBS, c = tid / kBS;
  const int b = b0 + bl;
  const int KLr = H / kKC;  // this thread's k range [c*KLr, (c+1)*KLr), a multiple of 4
  // the gate epilogue's operands
  const int eu = tid / kBS, ebb = tid - eu * kBS;
  const int ebi = b0 + ebb, ej = j0 + eu;
  const bool epi = tid < kHS * kBS && ebi < B;
  float ex_r = 0.f, ex_z = 0.f, ex_n = 0.f, eb_r = 0.f, eb_z = 0.f, eb_n = 0.f, ehp = 0.f;
  if (epi) {
    const float* xr = xp + (int64_t)ebi * xp_ld;
    ex_r = xr[ej];
    ex_z = xr[H + ej];
    ex_n = xr[2 * H + ej];
    eb_r = b_hh[ej];
    eb_z = b_hh[H + ej];
    eb_n = b_hh[2 * H + ej];
    ehp = h_prev ? h_prev[(int64_t)ebi * hp_ld + ej] : 0.0f;
  }
  const bool hv_ok = h_prev != nullptr;  // uniform: no h0 at step 0 means h = 0 (then W is read instead)
  const float* hrow = hv_ok ? h_prev + (int64_t)(b < B ? b : B - 1) * hp_ld + c * KLr : w_hh + c * KLr;  // rows >= B: never stored
  const int n4 = R * H / 4;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  for (int k0 = 0; k0 < KLr; k0 += 32) {
    float4 hv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int kk = k0 + 4 * q < KLr ? k0 + 4 * q : KLr - 4;
      hv[q] = *reinterpret_cast<const float4*>(hrow + kk);
      if (!hv_ok) hv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (k0 == 0) {
      // rows: gate g of unit u is W_hh row g*H + j0 + u
      for (int i0 = tid; i0 < n4; i0 += kWV * kNT) {
        float4 wv[kWV];
#pragma unroll
        for (int v = 0; v < kWV; ++v) {
          const int i = i0 + v * kNT < n4 ? i0 + v * kNT : n4 - 1;
          const int r = (4 * i) / H, k = 4 * i - r * H;
          const int g = r / kHS, u = r - g * kHS;
          wv[v] = *reinterpret_cast<const float4*>(w_hh + (int64_t)(g * H + j0 + u) * H + k);
        }
#pragma unroll
        for (int v = 0; v < kWV; ++v) {  // clamped indices rewrite the last element with its own value
          const int i = i0 + v * kNT < n4 ? i0 + v * kNT : n4 - 1;
          const int r = (4 * i) / H, k = 4 * i - r * H;
          *reinterpret_cast<float4*>(W + r * H + k) = wv[v];
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (k0 + 4 * q < KLr) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const float4 wv = *reinterpret_cast<const float4*>(W + r * H + c * KLr + k0 + 4 * q);
          acc[r] = fmaf(wv.x, hv[q].x, fmaf(wv.y, hv[q].y, fmaf(wv.z, hv[q].z, fmaf(wv.w, hv[q].w, acc[r]))));
        }
      }
    }
  }
  // the kG k-chunks of each wave (lanes bl, bl + kBS, ...) summed by lane exchange; group g keeps rows r % kG == g
#pragma unroll
  for (int m = kBS; m < 64; m <<= 1)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] += __shfl_xor(acc[r], m, 64);
  const int wv_id = tid >> 6, grp = (tid & 63) / kBS;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (r % kG == grp) part[(wv_id * R + r) * kBS + bl] = acc[r];
  __syncthreads();
  // gates for kHS units x kBS batch rows
  if (epi) {
    const int u = eu, bb = ebb;
    float hr = 0.f, hz = 0.f, hn = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      hr += part[(w * R + 0 * kHS + u) * kBS + bb];
      hz += part[(w * R + 1 * kHS + u) * kBS + bb];
      hn += part[(w * R + 2 * kHS + u) * kBS + bb];
    }
    const float r = sigmoidf_(ex_r + (hr + eb_r));
    const float z = sigmoidf_(ex_z + (hz + eb_z));
    const float n = tanhf(ex_n + r * (hn + eb_n));
    const float hn_t = (1.0f - z) * n + z * ehp;
    h_out[(int64_t)ebi * ho_ld + ej] = hn_t;
    if (h_copy) h_copy[(int64_t)ebi * H + ej] = hn_t;  // the last step's h_T, [B, H]
    if (save) {  // training: r, z, n and W_hn h + b_hn of this step, [4][B, T, H] (same row layout as h_out)
      float* sv = save + (int64_t)ebi * ho_ld + ej;
      sv[0] = r;
      sv[save_plane] = z;
      sv[2 * save_plane] = n;
      sv[3 * save_plane] = hn + eb_n;
    }
  }
}

// ---------------------------------------------------------------------------------------
// The recurrence as ONE persistent launch (hidden 512, batch <= 64): the per-step launches above pay a
// kernel boundary and re-stage their W_hh slice into LDS every step (7.4-7.8 us per step at config 2).
// Batch items are independent, so the 256 workgroups (one per CU) form 8 groups of 32; group g owns items
// g, g + 8, ... (<= 8 of them) and its slot s owns hidden units [16 s, 16 s + 16): the slot's 48 rows of
// W_hh (gates r, z, n) stay on-chip for the whole sequence.  A step needs the group's whole h_{t-1},
// written by its 32 slots: each slot stores its 16 units per item, drains them (s_waitcnt vmcnt(0)),
// joins a workgroup barrier, and ONE lane adds to the group's counter (agent-scope atomic); a slot starts
// step t once that counter reaches 32 t (one lane polls with sc1 loads, then a workgroup barrier) and
// reads h_{t-1} with sc1 loads (L1 bypassed) — MI355X_MICROARCH.md "Valid forms", hand-off table row 1.
// Where the groups live is decided at start by a census, not assumed: every workgroup reads its XCD
// (HW_REG_XCC_ID), takes a ticket on that XCD's arrival counter, then waits until all 256 have arrived.
//   * every XCD holds exactly 32 workgroups (the observed round-robin dispatch): group = XCD, slot =
//     ticket, and h stays in that XCD's L2 — plain (write-back) stores, L2-served sc1 loads;
//   * otherwise: group = blockIdx % 8, slot = blockIdx / 8, and h goes through memory — write-through
//     (sc1) stores — so any placement is correct, only slower.
// The h_t addresses are fresh every step (the output sequence), so no cache holds an older copy.  Every
// wait is bounded: a launch whose workgroups cannot all be resident at once sets an abort word and ends
// (garbage out) instead of hanging.  The slot's 48 rows of W_hh (gates r, z, n of its 16 units) live in
// REGISTERS for the whole sequence, split once into three bf16 terms (common.h split_bf16x3) as the A
// fragments of v_mfma_f32_16x16x32_bf16: wave w owns k in [64 w, 64 w + 64) — two 32-wide chunks — and per
// gate one 16 x 32 tile (rows = the slot's 16 units) per chunk.  Per step h_{t-1} of the group's items is
// staged once into LDS (16 KB); each wave splits its 64 k of the 8 items into B fragments (items are the
// tile's columns; columns 8-15 are zero) and runs 3 gates x 2 chunks x 6 products = 36 MFMAs — an
// fp32-accurate W_hh h — the 8 waves' partial sums meet in LDS and 128 epilogue threads apply the gates, one
// (item, unit) each.  (Per-step phases by in-kernel stamps, tools/exp_gru_clock.py: on the fp32 VALU — 384
// FMAs per lane plus a DPP and an LDS reduction — the compute phase took 1.9 us of a 3.7-3.8 us step,
// profiles/r06k_gruclk.log.)
constexpr int kPG = 8;             // groups (items g, g + 8, ... belong to group g)
constexpr int kPS = 32;            // slots per group
constexpr int kPU = 16;            // hidden units per slot (hidden = kPS * kPU = 512)
constexpr int kPH = kPS * kPU;
constexpr int kPR = 3 * kPU;       // W_hh rows per slot
constexpr int kPI = 8;             // items per group (batch <= kPG * kPI)
constexpr int kPCounterStride = 32;  // uint32 words between counters (one 128-B line each)
// sync words: [g * stride] step counter of group g; [(8 + x) * stride] arrivals on XCD x; [16 * stride] all
// arrivals; [17 * stride] abort; [18 * stride] route status (DDSP_HIP_GRU_STATUS_* bits, include/ddsp_hip.h)
constexpr int kPAbortWord = 17 * kPCounterStride;
constexpr int kPStatusWord = 18 * kPCounterStride;
constexpr int kPSyncWords = 19 * kPCounterStride;
constexpr uint64_t kPSpinTicks = 20000000;  // 200 ms at the 100 MHz realtime clock: an abort, never a hang

__device__ __forceinline__ float4 ld_sc1_f4(__amdgpu_buffer_rsrc_t r, int voff) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 16 /* sc1 */);
  return make_float4(__int_as_float(v.x), __int_as_float(v.y), __int_as_float(v.z), __int_as_float(v.w));
}

template <int AUX>
__device__ __forceinline__ void st_f4(__amdgpu_buffer_rsrc_t r, int voff, float4 v) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 x = {__float_as_int(v.x), __float_as_int(v.y), __float_as_int(v.z), __float_as_int(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(x, r, voff, 0, AUX);
}

// lane 0 waits until *word >= target (sc1 polls), bounded; false = aborted (by itself or another group)
__device__ __forceinline__ bool wait_at_least(uint32_t* word, uint32_t target, uint32_t* abort_word) {
  uint32_t n = 0;
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if ((++n & 63) == 0 && (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                            __builtin_amdgcn_s_memrealtime() - t_start > kPSpinTicks)) {
      __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// An aborted launch (a workgroup that could not be resident within kPSpinTicks: beside another long-running
// kernel, on a CU-masked stream, under GPU sharing) simply ends: every workgroup that sees the abort word
// returns.  The outputs are then recomputed by gru_rescue_kernel, which the same call enqueues behind the
// persistent launch and which does nothing unless the abort word is set — so the caller always gets the
// step kernels' values (bit for bit), never NaN or a half-finished sequence, and stream order (not a race
// between workgroups of one launch) decides which values survive.

template <bool kLocal>
__device__ __forceinline__ void gru_persistent_body(const float* __restrict__ xp, const float* __restrict__ w_hh,
                                                    const float* __restrict__ b_hh, const float* __restrict__ h0,
                                                    float* __restrict__ h_last, float* __restrict__ save, int B, int T,
                                                    int g, int s, uint32_t* __restrict__ counter,
                                                    uint32_t* __restrict__ abort_word, __amdgpu_buffer_rsrc_t rout,
                                                    float* hs, float (*part)[kPI][kPR], int* s_abort) {
  constexpr int kStoreAux = kLocal ? 0 : 16;  // write-back into the XCD's L2, or write-through (sc1)
  const int nI = B > g ? (B - g + kPG - 1) / kPG : 0;  // items of this group
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int q = l >> 4, l16 = l & 15;
  const int64_t item_stride = (int64_t)T * kPH;  // floats between items in out
  const int u0 = s * kPU;
  // this lane's A fragments: gate gt, chunk c: W_hh[gt * 512 + u0 + l16][64 w + 32 c + 8 q .. + 7], split
  u32x4_t wa[3][2][3];
#pragma unroll
  for (int gt = 0; gt < 3; ++gt)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float* src = w_hh + (int64_t)(gt * kPH + u0 + l16) * kPH + 64 * w + 32 * c + 8 * q;
      split_bf16x3(*reinterpret_cast<const float4*>(src), *reinterpret_cast<const float4*>(src + 4), wa[gt][c][0],
                   wa[gt][c][1], wa[gt][c][2]);
    }
  // epilogue role: e < 128 -> unit u0 + eu of item ei
  const int eu = tid & 15, ei = tid >> 4;
  const bool epi = tid < kPU * kPI && ei < nI;
  const int eb = g + kPG * ei;  // the epilogue item's batch index
  float ebr = 0.f, ebz = 0.f, ebn = 0.f, ehp = 0.f;
  if (epi) {
    ebr = b_hh[u0 + eu];
    ebz = b_hh[kPH + u0 + eu];
    ebn = b_hh[2 * kPH + u0 + eu];
    if (h0) ehp = h0[(int64_t)eb * kPH + u0 + eu];
  }
  // h staging role: thread -> item tid >> 6, floats 8 (tid & 63) .. + 7 of its 512
  const int hi = tid >> 6, hk = 8 * (tid & 63);
  const bool hok = hi < nI;
  const int hb = g + kPG * (hok ? hi : 0);
  for (int t = 0; t < T; ++t) {
    // the epilogue's input projection for this step: issued before the wait
    float exr = 0.f, exz = 0.f, exn = 0.f;
    if (epi) {
      const float* xr = xp + ((int64_t)eb * T + t) * 3 * kPH + u0 + eu;
      exr = xr[0];
      exz = xr[kPH];
      exn = xr[2 * kPH];
    }
    if (t > 0) {  // every slot of the group has published h_{t-1}
      if (tid == 0 && !wait_at_least(counter, (uint32_t)kPS * (uint32_t)t, abort_word)) *s_abort = 1;
      __syncthreads();
      if (*s_abort) return;  // gru_rescue_kernel recomputes the outputs
    }
    // h_{t-1} of the group's items into LDS, once per step (zeros past nI)
    {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (t > 0) {
        const int off = (int)(((int64_t)hb * item_stride + (int64_t)(t - 1) * kPH + hk) * 4);
        a = ld_sc1_f4(rout, off);
        b = ld_sc1_f4(rout, off + 16);
      } else if (h0) {
        a = *reinterpret_cast<const float4*>(h0 + (int64_t)hb * kPH + hk);
        b = *reinterpret_cast<const float4*>(h0 + (int64_t)hb * kPH + hk + 4);
      }
      if (!hok) a = b = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(&hs[hi * kPH + hk]) = a;
      *reinterpret_cast<float4*>(&hs[hi * kPH + hk + 4]) = b;
    }
    __syncthreads();
    // W_hh h_{t-1} for this wave's 64 k: item l16 (< 8; the other columns zero) is the tiles' column
    f32x4_t acc[3] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (l16 < kPI) {
        a = *reinterpret_cast<const float4*>(&hs[l16 * kPH + 64 * w + 32 * c + 8 * q]);
        b = *reinterpret_cast<const float4*>(&hs[l16 * kPH + 64 * w + 32 * c + 8 * q + 4]);
      }
      u32x4_t hb[3];
      split_bf16x3(a, b, hb[0], hb[1], hb[2]);
#pragma unroll
      for (int gt = 0; gt < 3; ++gt) {  // small terms first
        f32x4_t v = acc[gt];
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[gt][c][1]), as_bf16x8(hb[1]), v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[gt][c][2]), as_bf16x8(hb[0]), v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[gt][c][0]), as_bf16x8(hb[2]), v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[gt][c][1]), as_bf16x8(hb[0]), v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[gt][c][0]), as_bf16x8(hb[1]), v, 0, 0, 0);
        acc[gt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[gt][c][0]), as_bf16x8(hb[0]), v, 0, 0, 0);
      }
    }
    // acc[gt][e]: unit 4 q + e, item l16 -> part[w][item][gt * 16 + unit]
    if (l16 < kPI) {
#pragma unroll
      for (int gt = 0; gt < 3; ++gt)
        *reinterpret_cast<float4*>(&part[w][l16][gt * kPU + 4 * q]) =
            make_float4(acc[gt][0], acc[gt][1], acc[gt][2], acc[gt][3]);
    }
    __syncthreads();
    if (epi) {
      float hr = 0.f, hz = 0.f, hn = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) {  // over the 8 waves, fixed order
        hr += part[v][ei][eu];
        hz += part[v][ei][kPU + eu];
        hn += part[v][ei][2 * kPU + eu];
      }
      const float r = sigmoidf_(exr + (hr + ebr));
      const float z = sigmoidf_(exz + (hz + ebz));
      const float hbn = hn + ebn;
      const float n = tanhf(exn + r * hbn);
      const float hnew = (1.0f - z) * n + z * ehp;
      const int64_t oi = (int64_t)eb * item_stride + (int64_t)t * kPH + u0 + eu;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(hnew), rout, (int)(oi * 4), 0, kStoreAux);
      if (save) {
        const int64_t plane = (int64_t)B * T * kPH;
        save[oi] = r;
        save[plane + oi] = z;
        save[2 * plane + oi] = n;
        save[3 * plane + oi] = hbn;
      }
      if (h_last && t == T - 1) h_last[(int64_t)eb * kPH + u0 + eu] = hnew;
      ehp = hnew;
    }
    if (t + 1 < T) {  // publish h_t: drained stores, the workgroup's barrier, one agent-scope add
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ void __launch_bounds__(256) zero_words_kernel(uint32_t* __restrict__ w, int n) {
  for (int i = threadIdx.x; i < n; i += 256) w[i] = 0u;
}

// The persistent launches' start (forward and BPTT): this workgroup's XCD and its ticket there, then every
// workgroup's arrival (bounded: an abort, never a hang); the group / slot assignment and the hand-off form.
__device__ void persistent_census(uint32_t* __restrict__ sync, int flags, int* s_abort, int* s_local, int* s_group,
                                  int* s_slot) {
  uint32_t* abort_word = sync + kPAbortWord;
  if (threadIdx.x == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    const uint32_t ticket = __hip_atomic_fetch_add(sync + (kPG + xcc) * kPCounterStride, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    // (the ticket's value is used: the XCD add has completed before the total add)
    __hip_atomic_fetch_add(sync + 16 * kPCounterStride, ticket < 0x7fffffffu ? 1u : 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (flags & DDSP_HIP_GRU_FORCE_ABORT)  // test hook: the abort path without a residency failure
      __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = wait_at_least(sync + 16 * kPCounterStride, (uint32_t)(kPG * kPS), abort_word);
    // a workgroup whose census completed on its first poll has not looked at the abort word yet
    ok = ok && __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    int local = !(flags & DDSP_HIP_GRU_SPREAD);
    if (ok) {
      for (int x = 0; x < kPG; ++x)
        local &= __hip_atomic_load(sync + (kPG + x) * kPCounterStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 (uint32_t)kPS;
      if (blockIdx.x == 0)  // one writer: which hand-off the launch used
        __hip_atomic_store(sync + kPStatusWord, local ? (uint32_t)DDSP_HIP_GRU_STATUS_LOCAL : 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    *s_abort = !ok;
    *s_local = local;
    *s_group = local ? (int)xcc : (int)(blockIdx.x % kPG);
    *s_slot = local ? (int)ticket : (int)(blockIdx.x / kPG);
  }
  __syncthreads();
}

__global__ void __launch_bounds__(512) gru_persistent_kernel(
    const float* __restrict__ xp, const float* __restrict__ w_hh, const float* __restrict__ b_hh,
    const float* __restrict__ h0, float* __restrict__ out, float* __restrict__ h_last, float* __restrict__ save,
    int B, int T, uint32_t* __restrict__ sync, int flags) {
  __shared__ __attribute__((aligned(16))) float hs[kPI * kPH];      // h_{t-1} of the group's items, 16 KB
  __shared__ __attribute__((aligned(16))) float part[8][kPI][kPR];  // per-wave k partials [wave][item][row]
  __shared__ int s_abort, s_local, s_slot, s_group;
  uint32_t* abort_word = sync + kPAbortWord;
  persistent_census(sync, flags, &s_abort, &s_local, &s_group, &s_slot);
  __syncthreads();
  if (s_abort) return;  // gru_rescue_kernel recomputes the outputs
  const int g = s_group, s = s_slot;
  if (B <= g) return;  // the group has no items: nobody waits for it
  // out as a buffer resource: byte offsets (< 2^31, checked by the host) with cache-policy bits
  const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7fffffff, 0x00020000);
  uint32_t* counter = sync + g * kPCounterStride;
  if (s_local)
    gru_persistent_body<true>(xp, w_hh, b_hh, h0, h_last, save, B, T, g, s, counter, abort_word, rout, hs, part,
                              &s_abort);
  else
    gru_persistent_body<false>(xp, w_hh, b_hh, h0, h_last, save, B, T, g, s, counter, abort_word, rout, hs, part,
                               &s_abort);
}

// The persistent launch's rescue, enqueued right behind it on the same stream by every
// ddsp_hip_gru_forward_persistent call: unless the launch aborted it returns at once (one launch of B
// one-wave-instruction workgroups, ~2 us).  After an abort it recomputes out, h_last and gates with
// gru_step_kernel<16, 32, 512>'s arithmetic in the same order — each 16-wide k chunk's fma chain, the
// chunks summed in pairs, pairs of pairs, then over the 8 waves from zero — so the results equal the step
// kernels' bit for bit.  One workgroup per item (no residency requirement: the items are independent);
// a half-wave per W_hh row (lane c holds k chunk c, 64 contiguous bytes of the row), 16 rows per pass,
// W_hh re-read from L2 every step: slow (a fallback), but never wrong.
__global__ void __launch_bounds__(512) gru_rescue_kernel(const float* __restrict__ xp, const float* __restrict__ w_hh,
                                                         const float* __restrict__ b_hh, const float* __restrict__ h0,
                                                         float* __restrict__ out, float* __restrict__ h_last,
                                                         float* __restrict__ save, int B, int T,
                                                         uint32_t* __restrict__ sync) {
  if (__hip_atomic_load(sync + kPAbortWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
  __shared__ __attribute__((aligned(16))) float hs[kPH];  // h_{t-1} of this item
  __shared__ float rows[3 * kPH];                           // W_hh h_{t-1} per gate row
  const int tid = threadIdx.x, b = blockIdx.x;
  const int lane = tid & 63, c = lane & 31;  // k chunk c: [16 c, 16 c + 16)
  const int half = tid >> 5;                 // 16 half-waves
  float hp = h0 ? h0[(int64_t)b * kPH + tid] : 0.0f;  // this thread's unit in the epilogue
  hs[tid] = hp;
  const float br = b_hh[tid], bz = b_hh[kPH + tid], bn = b_hh[2 * kPH + tid];
  const int64_t plane = (int64_t)B * T * kPH;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    for (int row = half; row < 3 * kPH; row += 16) {
      const float* wrow = w_hh + (int64_t)row * kPH + 16 * c;
      float a = 0.0f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 w = *reinterpret_cast<const float4*>(wrow + 4 * q);
        const float4 h = *reinterpret_cast<const float4*>(&hs[16 * c + 4 * q]);
        a = fmaf(w.x, h.x, fmaf(w.y, h.y, fmaf(w.z, h.z, fmaf(w.w, h.w, a))));
      }
      // gru_step_kernel's lane exchanges (xor 16, then 32, over the wave's 4 k chunks) as xor 1, 2 here
      a += __shfl_xor(a, 1, 64);
      a += __shfl_xor(a, 2, 64);
      float s = 0.0f;
#pragma unroll
      for (int v = 0; v < 8; ++v) s += __shfl(a, (lane & 32) + 4 * v, 64);  // over its 8 waves, in order
      if (c == 0) rows[row] = s;
    }
    __syncthreads();
    const float* xr = xp + ((int64_t)b * T + t) * 3 * kPH;
    const float r = sigmoidf_(xr[tid] + (rows[tid] + br));
    const float z = sigmoidf_(xr[kPH + tid] + (rows[kPH + tid] + bz));
    const float hn = rows[2 * kPH + tid];
    const float n = tanhf(xr[2 * kPH + tid] + r * (hn + bn));
    hp = (1.0f - z) * n + z * hp;
    const int64_t oi = ((int64_t)b * T + t) * kPH + tid;
    out[oi] = hp;
    if (save) {
      save[oi] = r;
      save[plane + oi] = z;
      save[2 * plane + oi] = n;
      save[3 * plane + oi] = hn + bn;
    }
    hs[tid] = hp;  // every read of h_{t-1} (the row pass) is behind the barrier above
    __syncthreads();
  }
  if (h_last) h_last[(int64_t)b * kPH + tid] = hp;
  if (b == 0 && tid == 0)
    __hip_atomic_store(sync + kPStatusWord, (uint32_t)DDSP_HIP_GRU_STATUS_RESCUED, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------
// Backward (BPTT) of the recurrence, for training.  With dh the total gradient reaching h_t:
//   dn = dh (1 - z), dz = dh (h_{t-1} - n), da_n = dn (1 - n^2), da_z = dz z (1 - z),
//   da_r = da_n hn r (1 - r), dhn = da_n r     (hn = W_hn h_{t-1} + b_hn)
//   dxp_t = (da_r, da_z, da_n)   -> the input projection's gradient (GEMMs on the host side)
//   dG_t  = (da_r, da_z, dhn)    -> dW_hh = sum_t dG_t^T h_{t-1}, db_hh = sum_t dG_t (host GEMMs)
//   dh_{t-1} = dh z + W_hh^T dG_t + dout_{t-1}
// One launch per step: the transposed product for a slice of units x a batch tile, then, for the
// same (b, unit) elements, the step t-1 elementwise part (its dxp and dG_n) so the next launch
// finds dG_{t-1} ready.

// the elementwise part at step t for element (b, j), given the total dh: writes dxp, dGn
__device__ __forceinline__ void gru_bwd_elem_v(float r, float z, float n, float hn, int64_t idx, float hprev,
                                               float dh, float* __restrict__ dxp, int64_t xi, int H,
                                               float* __restrict__ dgn) {
  const float dn = dh * (1.0f - z);
  const float dz = dh * (hprev - n);
  const float dan = dn * (1.0f - n * n);
  const float daz = dz * z * (1.0f - z);
  const float dar = dan * hn * r * (1.0f - r);
  dxp[xi] = dar;
  dxp[xi + H] = daz;
  dxp[xi + 2 * H] = dan;
  dgn[idx] = dan * r;
}

__device__ __forceinline__ void gru_bwd_elem(const float* __restrict__ save, int64_t plane, int64_t idx, float hprev,
                                             float dh, float* __restrict__ dxp, int64_t xi, int H,
                                             float* __restrict__ dgn) {
  gru_bwd_elem_v(save[idx], save[plane + idx], save[2 * plane + idx], save[3 * plane + idx], idx, hprev, dh, dxp, xi,
                 H, dgn);
}

// WT[i][k] = W_hh[k][i] (H x 3H), so the backward's per-unit columns are contiguous rows; 32x32 tiles
__global__ void __launch_bounds__(256) transpose_kernel(const float* __restrict__ w, float* __restrict__ wt, int rows,
                                                        int cols) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8)
    if (r0 + y < rows && c0 + tx < cols) tile[y][tx] = w[(int64_t)(r0 + y) * cols + c0 + tx];
  __syncthreads();
  for (int y = ty; y < 32; y += 8)
    if (c0 + y < cols && r0 + tx < rows) wt[(int64_t)(c0 + y) * rows + r0 + tx] = tile[tx][y];
}

// step T-1's elementwise part from dh = dout[:, T-1] (+ dh_last); grid-stride over B*H
__global__ void gru_bwd_init_kernel(const float* __restrict__ dout, const float* __restrict__ dh_last,
                                    const float* __restrict__ out, const float* __restrict__ h0,
                                    const float* __restrict__ save, int64_t plane, float* __restrict__ dxp,
                                    float* __restrict__ dgn, float* __restrict__ dh_buf, int B, int T, int H) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)B * H;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / H, j = e - b * H;
    const int64_t idx = (b * T + (T - 1)) * H + j;
    float dh = dout ? dout[idx] : 0.0f;
    if (dh_last) dh += dh_last[e];
    const float hprev = T >= 2 ? out[idx - H] : (h0 ? h0[e] : 0.0f);
    dh_buf[e] = dh;
    gru_bwd_elem(save, plane, idx, hprev, dh, dxp, (b * T + (T - 1)) * 3 * H + j, H, dgn);
  }
}

// step t (>= 1): dh_{t-1} for units [i0, i0+kHS) x a batch tile, then step t-1's elementwise
// part; t == 0 writes dh0 only.  grid (H / kHS, ceil(B / kBS)); LDS: W_hh columns [3H][kHS] +
// per-wave partials [kNT / 64][kHS][kBS].  As in the forward step: every global load issued before
// the first wait (kH = 512 makes the loop bounds compile-time constants), the k-chunk partials
// summed inside each wave by lane exchanges.
template <int kBS, int kKC, int kH>
__global__ void __launch_bounds__(kBS * kKC) gru_bwd_step_kernel(
    const float* __restrict__ w_t, const float* __restrict__ save, int64_t plane, const float* __restrict__ dout,
    const float* __restrict__ out, const float* __restrict__ h0, float* __restrict__ dxp, float* __restrict__ dgn,
    const float* __restrict__ dh_in, float* __restrict__ dh_outbuf, float* __restrict__ dh0, int B, int T, int H_arg,
    int t) {
  extern __shared__ float smem[];
  constexpr int kNT = kBS * kKC;
  constexpr int kWaves = kNT / 64, kG = 64 / kBS;
  static_assert(kBS <= 64 && 64 % kBS == 0 && kNT % 64 == 0 && (kHS % kG == 0 || kG % kHS == 0), "tile shape");
  constexpr int kWV = 4;            // W columns' float4s per thread per staging round
  const int H = kH ? kH : H_arg;
  const int K = 3 * H;
  float* Wt = smem;                 // [K][kHS]: Wt[k][u] = W_hh[k][i0 + u]
  float* part = smem + K * kHS;     // [kWaves][kHS][kBS]
  const int i0 = blockIdx.x * kHS, b0 = blockIdx.y * kBS;
  const int tid = threadIdx.x;
  const int bl = tid % kBS, c = tid / kBS;
  const int b = b0 + bl;
  const int KLr = K / kKC;  // this thread's reduction range (K % (4 kKC) == 0)
  // the epilogue's operands (this step's z and dh, step t-1's saved gates, dout and h_{t-2})
  const int eu = tid / kBS, ebb = tid - eu * kBS;
  const int ebi = b0 + ebb, ei = i0 + eu;
  const bool epi = tid < kHS * kBS && ebi < B;
  const int64_t ee = (int64_t)ebi * H + ei;
  const int64_t eidx_t = ((int64_t)ebi * T + t) * H + ei, eidx = eidx_t - H;
  float e_dh = 0.f, e_z = 0.f, e_dout = 0.f, e_hprev = 0.f, s_r = 0.f, s_z = 0.f, s_n = 0.f, s_hn = 0.f;
  if (epi) {
    e_dh = dh_in[ee];
    e_z = save[plane + eidx_t];
    if (t > 0) {
      e_dout = dout ? dout[eidx] : 0.0f;
      e_hprev = t >= 2 ? out[eidx - H] : (h0 ? h0[ee] : 0.0f);
      s_r = save[eidx];
      s_z = save[plane + eidx];
      s_n = save[2 * plane + eidx];
      s_hn = save[3 * plane + eidx];
    }
  }
  // this thread's dG_t chunk [c KLr, (c+1) KLr) of row b (rows >= B read row B-1 and are never stored)
  const int bc = b < B ? b : B - 1;
  const float* gx = dxp + ((int64_t)bc * T + t) * 3 * H;  // [3H]: r, z rows are dG
  const float* gn = dgn + ((int64_t)bc * T + t) * H;      // [H]: dG_n
  const int k0 = c * KLr;
  const int n4 = kHS * K / 4;
  float acc[kHS];
#pragma unroll
  for (int u = 0; u < kHS; ++u) acc[u] = 0.0f;
  for (int kb = k0; kb < k0 + KLr; kb += 64) {
    float4 g4[16];  // 16 16-B loads before consuming them (the first batch overlaps the W staging)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = kb + 4 * q < k0 + KLr ? kb + 4 * q : k0 + KLr - 4;
      g4[q] = *reinterpret_cast<const float4*>(k < 2 * H ? gx + k : gn + (k - 2 * H));
    }
    if (kb == k0) {
      for (int e0 = tid; e0 < n4; e0 += kWV * kNT) {
        float4 wv[kWV];
#pragma unroll
        for (int v = 0; v < kWV; ++v) {
          const int e = e0 + v * kNT < n4 ? e0 + v * kNT : n4 - 1;
          const int u = e / (K / 4), k = 4 * (e - u * (K / 4));
          wv[v] = *reinterpret_cast<const float4*>(w_t + (int64_t)(i0 + u) * K + k);
        }
#pragma unroll
        for (int v = 0; v < kWV; ++v) {  // clamped indices rewrite the last element with its own value
          const int e = e0 + v * kNT < n4 ? e0 + v * kNT : n4 - 1;
          const int u = e / (K / 4), k = 4 * (e - u * (K / 4));
          Wt[(k + 0) * kHS + u] = wv[v].x;
          Wt[(k + 1) * kHS + u] = wv[v].y;
          Wt[(k + 2) * kHS + u] = wv[v].z;
          Wt[(k + 3) * kHS + u] = wv[v].w;
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = kb + 4 * q;
      if (k < k0 + KLr) {
        const float gv[4] = {g4[q].x, g4[q].y, g4[q].z, g4[q].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float4 w = *reinterpret_cast<const float4*>(Wt + (k + e) * kHS);
          acc[0] = fmaf(w.x, gv[e], acc[0]);
          acc[1] = fmaf(w.y, gv[e], acc[1]);
          acc[2] = fmaf(w.z, gv[e], acc[2]);
          acc[3] = fmaf(w.w, gv[e], acc[3]);
        }
      }
    }
  }
#pragma unroll
  for (int m = kBS; m < 64; m <<= 1)
#pragma unroll
    for (int u = 0; u < kHS; ++u) acc[u] += __shfl_xor(acc[u], m, 64);
  const int wv_id = tid >> 6, grp = (tid & 63) / kBS;
#pragma unroll
  for (int u = 0; u < kHS; ++u)
    if (u % kG == grp % kHS) part[(wv_id * kHS + u) * kBS + bl] = acc[u];
  __syncthreads();
  if (epi) {
    float s = 0.0f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += part[(w * kHS + eu) * kBS + ebb];
    // dh_{t-1} = dh_t z_t + W_hh^T dG_t + dout_{t-1}
    float dh = e_dh * e_z + s;
    if (t == 0) {
      if (dh0) dh0[ee] = dh;
    } else {
      dh += e_dout;
      dh_outbuf[ee] = dh;
      gru_bwd_elem_v(s_r, s_z, s_n, s_hn, eidx, e_hprev, dh, dxp, ((int64_t)ebi * T + (t - 1)) * 3 * H + ei, H, dgn);
    }
  }
}

// The backward step on the fp32 matrix cores (H = 512, steps t >= 2 with grad_out given; the other
// steps run gru_bwd_step_kernel): dh_{t-1} for 16 units x 16 batch rows is a 16 x 16 GEMM over
// K = 3H (A: dG_t rows, B: W_hh^T rows from the transposed copy), the K range split over the 8
// waves, every load issued before the first wait (as in the forward); then, for the same 256
// (b, unit) elements, step t-1's elementwise part.
constexpr int kBwdUnits = 16;
template <int kH>
__global__ void __launch_bounds__(512) gru_bwd_step_mfma_kernel(
    const float* __restrict__ w_t, const float* __restrict__ save, int64_t plane, const float* __restrict__ dout,
    const float* __restrict__ out, float* __restrict__ dxp, float* __restrict__ dgn, const float* __restrict__ dh_in,
    float* __restrict__ dh_outbuf, int B, int T, int t) {
  constexpr int H = kH, K = 3 * H, kKW = K / 8, kCh = kKW / 16;
  static_assert(H % 128 == 0, "tile shape");
  __shared__ float part[8][16][17];  // [wave][batch row][unit]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int q = lane >> 4, l16 = lane & 15;
  const int i0 = blockIdx.x * kBwdUnits, b0 = blockIdx.y * 16;
  // the epilogue's operands (threads < 256 store unit tid / 16 of batch row tid % 16; all load)
  const int eu = (tid >> 4) & 15, ebb = tid & 15;
  const int ebi = b0 + ebb < B ? b0 + ebb : B - 1, ei = i0 + eu;
  const bool epi = tid < kBwdUnits * 16 && b0 + ebb < B;
  const int64_t ee = (int64_t)ebi * H + ei;
  const int64_t eidx_t = ((int64_t)ebi * T + t) * H + ei, eidx = eidx_t - H;
  const float e_dh = dh_in[ee], e_z = save[plane + eidx_t], e_dout = dout[eidx], e_hprev = out[eidx - H];
  const float s_r = save[eidx], s_z = save[plane + eidx], s_n = save[2 * plane + eidx], s_hn = save[3 * plane + eidx];
  const int bA = b0 + l16 < B ? b0 + l16 : B - 1;  // rows >= B: loaded, never stored
  const float* gx = dxp + ((int64_t)bA * T + t) * 3 * H;  // [3H]: r, z rows are dG
  const float* gn = dgn + ((int64_t)bA * T + t) * H;      // [H]: dG_n
  const float* wrow = w_t + (int64_t)(i0 + l16) * K;
  float4 ga[kCh], wb[kCh];
#pragma unroll
  for (int c = 0; c < kCh; ++c) {
    const int k = wv * kKW + 16 * c + 4 * q;
    ga[c] = *reinterpret_cast<const float4*>(k < 2 * H ? gx + k : gn + (k - 2 * H));
    wb[c] = *reinterpret_cast<const float4*>(wrow + k);
  }
  __builtin_amdgcn_sched_barrier(0);  // every load above is issued before the first MFMA waits
  f32x4_t acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int c = 0; c < kCh; ++c) {
    acc[c & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[c].x, wb[c].x, acc[c & 1], 0, 0, 0);
    acc[c & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[c].y, wb[c].y, acc[c & 1], 0, 0, 0);
    acc[c & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[c].z, wb[c].z, acc[c & 1], 0, 0, 0);
    acc[c & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[c].w, wb[c].w, acc[c & 1], 0, 0, 0);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) part[wv][4 * q + e][l16] = acc[0][e] + acc[1][e];
  asm volatile("" ::"v"(e_dh), "v"(e_z), "v"(e_dout), "v"(e_hprev), "v"(s_r), "v"(s_z), "v"(s_n),
               "v"(s_hn));  // loads stay above the barrier
  __syncthreads();
  float sum = 0.0f;
#pragma unroll
  for (int w = 0; w < 8; ++w) sum += part[w][ebb][eu];
  // dh_{t-1} = dh_t z_t + W_hh^T dG_t + dout_{t-1}
  const float dh = e_dh * e_z + sum + e_dout;
  if (epi) {
    dh_outbuf[ee] = dh;
    gru_bwd_elem_v(s_r, s_z, s_n, s_hn, eidx, e_hprev, dh, dxp, ((int64_t)ebi * T + (t - 1)) * 3 * H + ei, H, dgn);
  }
}

// ---------------------------------------------------------------------------------------
// The BPTT as ONE persistent launch (hidden 512, batch <= 64; the training forward's mirror): the per-step
// backward launches above pay a kernel boundary and re-stage W_hh every step (9.7 us per step at config 2,
// 1.9 ms per layer).  Same groups, slots, census, hand-off and abort as the forward: slot s owns units
// [16 s, 16 s + 16) of its group's 8 items and keeps its W_hh columns — the A fragments of W_hh^T (rows =
// its 16 units, k = the 1536 gate rows; wave w owns k in [192 w, 192 w + 192), six 32-wide chunks), split
// into three bf16 terms — in registers.  Per step t (T-1 down to 0): wait until every slot has published
// dG_t = (da_r, da_z, dan r) — the grad_xp / grad_gn rows of step t themselves —, stage the group's 8 x 1536
// values into LDS (48 KB), W_hh^T dG_t for the slot's units on the bf16 matrix cores (36 MFMAs per wave,
// fp32-accurate), the 8 waves' partials through LDS, then 128 epilogue threads (unit, item):
// dh_{t-1} = dh_t z_t + W_hh^T dG_t + dout_{t-1} and step t-1's elementwise part (its dG, written and
// published); at t = 0 the last sums give dh0.  An abort (residency) leaves the outputs to
// gru_bwd_rescue_kernel, enqueued behind it.
__global__ void __launch_bounds__(512) gru_bptt_persistent_kernel(
    const float* __restrict__ w_hh, const float* __restrict__ save, const float* __restrict__ out,
    const float* __restrict__ h0, const float* __restrict__ dout, const float* __restrict__ dh_last,
    float* __restrict__ dxp, float* __restrict__ dgn, float* __restrict__ dh0, int B, int T,
    uint32_t* __restrict__ sync, int flags) {
  constexpr int K3 = 3 * kPH;  // 1536 gate rows
  __shared__ __attribute__((aligned(16))) float gs[kPI * K3];        // dG_t of the group's items, 48 KB
  __shared__ __attribute__((aligned(16))) float part[8][kPI][kPU];   // per-wave partials [wave][item][unit]
  __shared__ int s_abort, s_local, s_slot, s_group;
  uint32_t* abort_word = sync + kPAbortWord;
  persistent_census(sync, flags, &s_abort, &s_local, &s_group, &s_slot);
  if (s_abort) return;  // gru_bwd_rescue_kernel recomputes the outputs
  const int g = s_group, s = s_slot;
  if (B <= g) return;
  const bool local = s_local;
  uint32_t* counter = sync + g * kPCounterStride;
  const int nI = (B - g + kPG - 1) / kPG;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int q = l >> 4, l16 = l & 15;
  const int u0 = s * kPU;
  const int64_t plane = (int64_t)B * T * kPH;
  // dxp / dgn as buffer resources (byte offsets < 2^31, checked by the host): the hand-off stores
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(dxp, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(dgn, (short)0, 0x7fffffff, 0x00020000);
  // A fragments: chunk c, lane (q, l16): W_hh[192 w + 32 c + 8 q + j][u0 + l16], j = 0..7, split
  u32x4_t wa[6][3];
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    const float* src = w_hh + (int64_t)(192 * w + 32 * c + 8 * q) * kPH + u0 + l16;
    const float4 a = make_float4(src[0], src[kPH], src[2 * kPH], src[3 * kPH]);
    const float4 b = make_float4(src[4 * kPH], src[5 * kPH], src[6 * kPH], src[7 * kPH]);
    split_bf16x3(a, b, wa[c][0], wa[c][1], wa[c][2]);
  }
  // epilogue role: tid < 128 -> unit u0 + eu of item ei
  const int eu = tid & 15, ei = tid >> 4;
  const bool epi = tid < kPU * kPI && ei < nI;
  const int eb = g + kPG * ei;
  const int j = u0 + eu;
  // the elementwise part of step t for this (item, unit) from its saved gates and h_{t-1} (loaded ahead by
  // load_elem): dG_t into dxp / dgn (write-back stores into the XCD's L2 on the local hand-off,
  // write-through otherwise)
  struct Elem { float r, z, n, hn, hprev, dout; };
  auto load_elem = [&](int t) -> Elem {
    const int64_t idx = ((int64_t)eb * T + t) * kPH + j;
    Elem e;
    e.r = save[idx];
    e.z = save[plane + idx];
    e.n = save[2 * plane + idx];
    e.hn = save[3 * plane + idx];
    e.hprev = t >= 1 ? out[idx - kPH] : (h0 ? h0[(int64_t)eb * kPH + j] : 0.0f);
    e.dout = dout ? dout[idx] : 0.0f;
    return e;
  };
  auto elem = [&](int t, float dh, const Elem& ev) {
    const int64_t idx = ((int64_t)eb * T + t) * kPH + j;
    const float r = ev.r, z = ev.z, n = ev.n, hn = ev.hn, hprev = ev.hprev;
    const float dn = dh * (1.0f - z);
    const float dz = dh * (hprev - n);
    const float dan = dn * (1.0f - n * n);
    const float daz = dz * z * (1.0f - z);
    const float dar = dan * hn * r * (1.0f - r);
    const int xo = (int)((((int64_t)eb * T + t) * 3 * kPH + j) * 4);
    const int go = (int)(idx * 4);
    if (local) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(dar), rx, xo, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(daz), rx, xo + 4 * kPH, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(dan), rx, xo + 8 * kPH, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(dan * r), rg, go, 0, 0);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(dar), rx, xo, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(daz), rx, xo + 4 * kPH, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(dan), rx, xo + 8 * kPH, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(dan * r), rg, go, 0, 16);
    }
  };
  float dh = 0.0f, zt = 0.0f;
  if (epi) {  // step T-1: dh = dout_{T-1} + dh_last
    const Elem ev = load_elem(T - 1);
    dh = ev.dout + (dh_last ? dh_last[(int64_t)eb * kPH + j] : 0.0f);
    zt = ev.z;
    elem(T - 1, dh, ev);
  }
  // staging role: thread -> item tid >> 6, 24 floats (6 float4) at 24 (tid & 63) .. of its 1536
  const int si = tid >> 6, sk = 24 * (tid & 63);
  const bool sok = si < nI;
  const int sb = g + kPG * (sok ? si : 0);
  for (int t = T - 1; t >= 0; --t) {
    // publish dG_t (written by this workgroup's epilogue threads): drained stores, barrier, one add
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!wait_at_least(counter, (uint32_t)kPS * (uint32_t)(T - t), abort_word)) s_abort = 1;
    }
    Elem ev{};  // step t-1's elementwise operands: issued before the wait completes
    if (epi && t >= 1) ev = load_elem(t - 1);
    __syncthreads();
    if (s_abort) return;
    // dG_t of the group's items into LDS (zeros past nI)
#pragma unroll
    for (int v = 0; v < 6; ++v) {
      const int k = sk + 4 * v;  // 4 consecutive gate rows, never crossing the 512-row gate planes
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      if (sok) {
        if (k < 2 * kPH) a = ld_sc1_f4(rx, (int)((((int64_t)sb * T + t) * 3 * kPH + k) * 4));
        else a = ld_sc1_f4(rg, (int)((((int64_t)sb * T + t) * kPH + (k - 2 * kPH)) * 4));
      }
      *reinterpret_cast<float4*>(&gs[si * K3 + k]) = a;
    }
    __syncthreads();
    // W_hh^T dG_t: units (rows) x items (columns 0..7; 8..15 zero)
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (l16 < kPI) {
        a = *reinterpret_cast<const float4*>(&gs[l16 * K3 + 192 * w + 32 * c + 8 * q]);
        b = *reinterpret_cast<const float4*>(&gs[l16 * K3 + 192 * w + 32 * c + 8 * q + 4]);
      }
      u32x4_t gb[3];
      split_bf16x3(a, b, gb[0], gb[1], gb[2]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[c][1]), as_bf16x8(gb[1]), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[c][2]), as_bf16x8(gb[0]), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[c][0]), as_bf16x8(gb[2]), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[c][1]), as_bf16x8(gb[0]), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[c][0]), as_bf16x8(gb[1]), acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wa[c][0]), as_bf16x8(gb[0]), acc, 0, 0, 0);
    }
    if (l16 < kPI)  // acc[e]: unit 4 q + e, item l16
      *reinterpret_cast<float4*>(&part[w][l16][4 * q]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    __syncthreads();
    if (epi) {
      float sum = 0.0f;
#pragma unroll
      for (int v = 0; v < 8; ++v) sum += part[v][ei][eu];  // over the 8 waves, fixed order
      const float dprev = dh * zt + sum;  // dh_{t-1} without dout_{t-1}
      if (t >= 1) {
        dh = dprev + ev.dout;
        zt = ev.z;
        elem(t - 1, dh, ev);
      } else if (dh0) {
        dh0[(int64_t)eb * kPH + j] = dprev;
      }
    }
  }
}

// The BPTT launch's rescue (as gru_rescue_kernel for the forward): nothing unless the launch aborted; then
// one workgroup per item redoes the whole BPTT, thread = unit, W_hh^T dG_t read from global memory row by
// row (coalesced over the units) — slow, never wrong.  fp32 sums in gate-row order.
__global__ void __launch_bounds__(512) gru_bwd_rescue_kernel(
    const float* __restrict__ w_hh, const float* __restrict__ save, const float* __restrict__ out,
    const float* __restrict__ h0, const float* __restrict__ dout, const float* __restrict__ dh_last,
    float* __restrict__ dxp, float* __restrict__ dgn, float* __restrict__ dh0, int B, int T,
    uint32_t* __restrict__ sync) {
  if (__hip_atomic_load(sync + kPAbortWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
  constexpr int K3 = 3 * kPH;
  __shared__ float gs[K3];  // dG_t of this item
  const int b = blockIdx.x, j = threadIdx.x;
  const int64_t plane = (int64_t)B * T * kPH;
  auto elem = [&](int t, float dh) -> float {
    const int64_t idx = ((int64_t)b * T + t) * kPH + j;
    const float r = save[idx], z = save[plane + idx], n = save[2 * plane + idx], hn = save[3 * plane + idx];
    const float hprev = t >= 1 ? out[idx - kPH] : (h0 ? h0[(int64_t)b * kPH + j] : 0.0f);
    const float dn = dh * (1.0f - z);
    const float dz = dh * (hprev - n);
    const float dan = dn * (1.0f - n * n);
    const float daz = dz * z * (1.0f - z);
    const float dar = dan * hn * r * (1.0f - r);
    const int64_t xi = ((int64_t)b * T + t) * 3 * kPH + j;
    dxp[xi] = dar;
    dxp[xi + kPH] = daz;
    dxp[xi + 2 * kPH] = dan;
    dgn[idx] = dan * r;
    gs[j] = dar;
    gs[kPH + j] = daz;
    gs[2 * kPH + j] = dan * r;
    return z;
  };
  float dh = (dout ? dout[((int64_t)b * T + (T - 1)) * kPH + j] : 0.0f) + (dh_last ? dh_last[(int64_t)b * kPH + j] : 0.0f);
  float zt = elem(T - 1, dh);
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    float sum = 0.0f;
    for (int r = 0; r < K3; ++r) sum = fmaf(w_hh[(int64_t)r * kPH + j], gs[r], sum);
    __syncthreads();  // every read of gs done before step t-1's elementwise part rewrites it
    const float dprev = dh * zt + sum;
    if (t >= 1) {
      dh = dprev + (dout ? dout[((int64_t)b * T + (t - 1)) * kPH + j] : 0.0f);
      zt = elem(t - 1, dh);
      __syncthreads();
    } else if (dh0) {
      dh0[(int64_t)b * kPH + j] = dprev;
    }
  }
  if (b == 0 && j == 0)
    __hip_atomic_store(sync + kPStatusWord, (uint32_t)DDSP_HIP_GRU_STATUS_RESCUED, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace
}  // namespace ddsp

using namespace ddsp;

extern "C" {

}  // extern "C"

// false when the stream's CU mask leaves out some of the device's cus CUs (a query failure counts as all)
static bool stream_reaches_all_cus(hipStream_t st, int cus) {
  uint32_t mask[32] = {0};
  const int words = (cus + 31) / 32;
  if (words > 32 || hipExtStreamGetCUMask(st, (uint32_t)words, mask) != hipSuccess) return true;
  int on = 0;
  for (int c = 0; c < cus; ++c) on += (mask[c >> 5] >> (c & 31)) & 1u;
  return on >= cus;
}

template <int kBS, int kKC, int kH = 0>
static int gru_backward_steps(const float* w_t, const float* gates, int64_t plane, const float* grad_out, const float* out,
                              const float* h0, float* grad_xp, float* grad_gn, float* const* dhb, float* grad_h0, int B,
                              int T, int H, hipStream_t st) {
  const size_t shm = sizeof(float) * ((size_t)3 * H * kHS + (size_t)(kBS * kKC / 64) * kHS * kBS);
  const dim3 grid((unsigned)(H / kHS), (unsigned)((B + kBS - 1) / kBS));
  for (int t = T - 1; t >= 0; --t) {
    hipLaunchKernelGGL((gru_bwd_step_kernel<kBS, kKC, kH>), grid, dim3(kBS * kKC), shm, st, w_t, gates, plane, grad_out, out,
                       h0, grad_xp, grad_gn, dhb[t & 1], dhb[(t - 1) & 1], grad_h0, B, T, H, t);
    int r = launch_status();
    if (r) return r;
  }
  return DDSP_HIP_OK;
}

template <int kBS, int kKC, int kH = 0>
static int gru_forward_launch(const float* xp, const float* w_hh, const float* b_hh, const float* h0, float* out,
                              float* h_last, float* gates, int64_t batch, int64_t steps, int64_t hidden, void* stream) {
  if (batch > 65535 * kBS) return DDSP_HIP_ERANGE;
  const int H = (int)hidden, B = (int)batch;
  const size_t shm = sizeof(float) * ((size_t)3 * kHS * H + (size_t)(kBS * kKC / 64) * 3 * kHS * kBS);
  const dim3 grid((unsigned)(H / kHS), (unsigned)((B + kBS - 1) / kBS));
  const int64_t row = steps * hidden;  // out[b] row stride: [B, T, H]
  // h_T goes to h_last from the last step's kernel, unless that step still reads h0 = h_last
  const bool direct = h_last && steps > 1;
  for (int64_t t = 0; t < steps; ++t) {
    const float* hp = t == 0 ? h0 : out + (t - 1) * hidden;
    const int64_t hp_ld = t == 0 ? hidden : row;
    hipLaunchKernelGGL((gru_step_kernel<kBS, kKC, kH>), grid, dim3(kBS * kKC), shm, reinterpret_cast<hipStream_t>(stream),
                       xp + t * 3 * hidden, w_hh, b_hh, hp, hp_ld, out + t * hidden, row, B, H, steps * 3 * hidden,
                       gates ? gates + t * hidden : nullptr, batch * steps * hidden,
                       direct && t == steps - 1 ? h_last : nullptr);
    int st = launch_status();
    if (st) return st;
  }
  if (h_last && !direct) {
    hipError_t e = hipMemcpy2DAsync(h_last, sizeof(float) * hidden, out + (steps - 1) * hidden, sizeof(float) * row,
                                    sizeof(float) * hidden, batch, hipMemcpyDeviceToDevice,
                                    reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) return DDSP_HIP_ELAUNCH;
  }
  return DDSP_HIP_OK;
}

extern "C" {

size_t ddsp_hip_gru_persistent_workspace_size(void) { return sizeof(uint32_t) * kPSyncWords; }

size_t ddsp_hip_gru_persistent_status_offset(void) { return sizeof(uint32_t) * kPStatusWord; }

int ddsp_hip_gru_forward_persistent(const float* xp, const float* w_hh, const float* b_hh, const float* h0, float* out,
                                    float* h_last, float* gates, int64_t batch, int64_t steps, int64_t hidden,
                                    int flags, void* workspace, size_t workspace_bytes, void* stream) {
  if (flags & ~(DDSP_HIP_GRU_SPREAD | DDSP_HIP_GRU_NO_MASK_CHECK | DDSP_HIP_GRU_FORCE_ABORT)) return DDSP_HIP_EINVAL;
  if (batch < 0 || steps < 0 || hidden < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || steps == 0) return DDSP_HIP_OK;
  if (!xp || !w_hh || !b_hh || !out) return DDSP_HIP_EINVAL;
  if (hidden != kPH || batch > kPG * kPI || batch * steps * hidden * (int64_t)sizeof(float) >= ((int64_t)1 << 31) ||
      steps > (int64_t)INT32_MAX / kPS)
    return DDSP_HIP_ERANGE;
  if (!workspace || workspace_bytes < ddsp_hip_gru_persistent_workspace_size()) return DDSP_HIP_EWORKSPACE;
  const uintptr_t al = reinterpret_cast<uintptr_t>(xp) | reinterpret_cast<uintptr_t>(w_hh) |
                       reinterpret_cast<uintptr_t>(b_hh) | reinterpret_cast<uintptr_t>(out) |
                       reinterpret_cast<uintptr_t>(h0) | reinterpret_cast<uintptr_t>(h_last) |
                       reinterpret_cast<uintptr_t>(gates);
  if (al & 15) return DDSP_HIP_ERANGE;
  // h_T over h0 in place: the groups finish independently, and a rescue after one group's abort re-reads h0
  if (h0 && h0 == h_last) return DDSP_HIP_ERANGE;
  // every workgroup of a group must be resident at once (237 VGPRs x 8 waves: one workgroup per CU)
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return DDSP_HIP_ELAUNCH;
  if (cus < kPG * kPS) return DDSP_HIP_ERANGE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // a stream whose kernels cannot reach every CU (hipExtStreamCreateWithCUMask, e.g. this library's
  // ddsp_hip_stream_create_cu_masked) cannot hold the grid: refuse up front rather than wait for the abort
  if (!(flags & DDSP_HIP_GRU_NO_MASK_CHECK) && !stream_reaches_all_cus(st, cus)) return DDSP_HIP_ERANGE;
  uint32_t* sync = reinterpret_cast<uint32_t*>(workspace);
  // the sync words are zeroed by a kernel of ours: a hipMemsetAsync captured into a HIP graph wrote
  // 0x5EE0B080 instead of 0 on every replay after the first (ROCm 7.2, tools/dbg_gru_graph.py)
  hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(256), 0, st, sync, kPSyncWords);
  if (int r = launch_status()) return r;
  hipLaunchKernelGGL(gru_persistent_kernel, dim3(kPG * kPS), dim3(512), 0, st, xp, w_hh, b_hh, h0, out, h_last, gates,
                     (int)batch, (int)steps, sync, flags);
  if (int r = launch_status()) return r;
  hipLaunchKernelGGL(gru_rescue_kernel, dim3((unsigned)batch), dim3(512), 0, st, xp, w_hh, b_hh, h0, out, h_last, gates,
                     (int)batch, (int)steps, sync);
  return launch_status();
}

int ddsp_hip_gru_forward(const float* xp, const float* w_hh, const float* b_hh, const float* h0, float* out,
                         float* h_last, float* gates, int64_t batch, int64_t steps, int64_t hidden, void* stream) {
  if (batch < 0 || steps < 0 || hidden < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || steps == 0) return DDSP_HIP_OK;
  if (!xp || !w_hh || !b_hh || !out) return DDSP_HIP_EINVAL;
  if (hidden % 64 || hidden > 4096) return DDSP_HIP_ERANGE;
  if (hidden == 512)  // the decoder's: compile-time bounds (a matrix-core form measured 8.5 vs 7.4-7.8 us per step)
    return gru_forward_launch<16, 32, 512>(xp, w_hh, b_hh, h0, out, h_last, gates, batch, steps, hidden, stream);
  if (hidden % 128 == 0)
    return gru_forward_launch<16, 32>(xp, w_hh, b_hh, h0, out, h_last, gates, batch, steps, hidden, stream);
  return gru_forward_launch<32, 16>(xp, w_hh, b_hh, h0, out, h_last, gates, batch, steps, hidden, stream);
}

int ddsp_hip_gru_backward_persistent(const float* w_hh, const float* gates, const float* out, const float* h0,
                                     const float* grad_out, const float* grad_h_last, float* grad_xp, float* grad_gn,
                                     float* grad_h0, int64_t batch, int64_t steps, int64_t hidden, int flags,
                                     void* workspace, size_t workspace_bytes, void* stream) {
  if (flags & ~(DDSP_HIP_GRU_SPREAD | DDSP_HIP_GRU_NO_MASK_CHECK | DDSP_HIP_GRU_FORCE_ABORT)) return DDSP_HIP_EINVAL;
  if (batch < 0 || steps < 0 || hidden < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || steps == 0) return DDSP_HIP_OK;
  if (!w_hh || !gates || !out || !grad_xp || !grad_gn) return DDSP_HIP_EINVAL;
  if (hidden != kPH || batch > kPG * kPI || batch * steps * 3 * hidden * (int64_t)sizeof(float) >= ((int64_t)1 << 31) ||
      steps > (int64_t)INT32_MAX / kPS)
    return DDSP_HIP_ERANGE;
  if (!workspace || workspace_bytes < ddsp_hip_gru_persistent_workspace_size()) return DDSP_HIP_EWORKSPACE;
  if ((reinterpret_cast<uintptr_t>(grad_xp) | reinterpret_cast<uintptr_t>(grad_gn)) & 15) return DDSP_HIP_ERANGE;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return DDSP_HIP_ELAUNCH;
  if (cus < kPG * kPS) return DDSP_HIP_ERANGE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (!(flags & DDSP_HIP_GRU_NO_MASK_CHECK) && !stream_reaches_all_cus(st, cus)) return DDSP_HIP_ERANGE;
  uint32_t* sync = reinterpret_cast<uint32_t*>(workspace);
  hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(256), 0, st, sync, kPSyncWords);
  if (int r = launch_status()) return r;
  hipLaunchKernelGGL(gru_bptt_persistent_kernel, dim3(kPG * kPS), dim3(512), 0, st, w_hh, gates, out, h0, grad_out,
                     grad_h_last, grad_xp, grad_gn, grad_h0, (int)batch, (int)steps, sync, flags);
  if (int r = launch_status()) return r;
  hipLaunchKernelGGL(gru_bwd_rescue_kernel, dim3((unsigned)batch), dim3(512), 0, st, w_hh, gates, out, h0, grad_out,
                     grad_h_last, grad_xp, grad_gn, grad_h0, (int)batch, (int)steps, sync);
  return launch_status();
}

size_t ddsp_hip_gru_backward_workspace_size(int64_t batch, int64_t hidden) {
  if (batch < 1 || hidden < 1) return 0;
  return sizeof(float) * ((size_t)2 * batch * hidden + (size_t)3 * hidden * hidden);
}

int ddsp_hip_gru_backward(const float* w_hh, const float* gates, const float* out, const float* h0,
                          const float* grad_out, const float* grad_h_last, float* grad_xp, float* grad_gn,
                          float* grad_h0, int64_t batch, int64_t steps, int64_t hidden, void* workspace,
                          size_t workspace_bytes, void* stream) {
  if (batch < 0 || steps < 0 || hidden < 1) return DDSP_HIP_EINVAL;
  if (batch == 0 || steps == 0) return DDSP_HIP_OK;
  if (!w_hh || !gates || !out || !grad_xp || !grad_gn) return DDSP_HIP_EINVAL;
  if (hidden % 64 || hidden > 4096 || batch > 65535 * 16) return DDSP_HIP_ERANGE;
  if (!workspace || workspace_bytes < ddsp_hip_gru_backward_workspace_size(batch, hidden)) return DDSP_HIP_EWORKSPACE;
  const int H = (int)hidden, B = (int)batch, T = (int)steps;
  const int64_t plane = batch * steps * hidden;
  float* dhb[2] = {reinterpret_cast<float*>(workspace), reinterpret_cast<float*>(workspace) + batch * hidden};
  float* w_t = reinterpret_cast<float*>(workspace) + 2 * batch * hidden;  // [H][3H]
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((H + 31) / 32), (unsigned)((3 * H + 31) / 32)), dim3(256), 0,
                     st, w_hh, w_t, 3 * H, H);
  const unsigned g1 = (unsigned)std::min<int64_t>((batch * hidden + 255) / 256, 65535);
  hipLaunchKernelGGL(gru_bwd_init_kernel, dim3(g1), dim3(256), 0, st, grad_out, grad_h_last, out, h0, gates, plane,
                     grad_xp, grad_gn, dhb[(T - 1) & 1], B, T, H);
  int r = launch_status();
  if (r) return r;
  if (H == 512 && grad_out) {  // steps t >= 2 on the MFMA kernel, t = 1, 0 (h0 / dh0 cases) on the generic one
    const dim3 grid((unsigned)(512 / kBwdUnits), (unsigned)((B + 15) / 16));
    const dim3 grid1((unsigned)(512 / kHS), (unsigned)((B + 15) / 16));
    const size_t shm1 = sizeof(float) * ((size_t)3 * 512 * kHS + (size_t)(16 * 32 / 64) * kHS * 16);
    for (int t = T - 1; t >= 0; --t) {
      if (t >= 2)
        hipLaunchKernelGGL(gru_bwd_step_mfma_kernel<512>, grid, dim3(512), 0, st, w_t, gates, plane, grad_out, out,
                           grad_xp, grad_gn, dhb[t & 1], dhb[(t - 1) & 1], B, T, t);
      else
        hipLaunchKernelGGL((gru_bwd_step_kernel<16, 32, 0>), grid1, dim3(512), shm1, st, w_t, gates, plane, grad_out,
                           out, h0, grad_xp, grad_gn, dhb[t & 1], dhb[(t - 1) & 1], grad_h0, B, T, H, t);
      if ((r = launch_status())) return r;
    }
  } else if (H % 128 == 0) {
    if ((r = gru_backward_steps<16, 32>(w_t, gates, plane, grad_out, out, h0, grad_xp, grad_gn, dhb, grad_h0, B, T, H, st)))
      return r;
  } else if ((r = gru_backward_steps<32, 16>(w_t, gates, plane, grad_out, out, h0, grad_xp, grad_gn, dhb, grad_h0, B, T,
                                             H, st))) {
    return r;
  }
  return DDSP_HIP_OK;
}

}  // extern "C"
