// embedding.hip — embedding row gather (fwd) and deterministic sparse Adagrad (bwd + update).
//
// Forward replaces keras.layers.Embedding (src/models.py:71,74): a pure row copy, HBM-bound.
// For D = 32/64/128 a wave loads the ids of RPW rows with one instruction (one per lane), then
// issues every row load of the batch before any store (D = 128: 2 rows of 512 B per wave
// instruction, RPW/2 instructions = 16-32 KB in flight per wave), the row id broadcast from its
// lane. A/B on the C3 user table (tools/ab_gather.py): 5.6 TB/s at 65,536 rows (RPW = 32),
// 6.0 TB/s at 1M rows (RPW = 64), vs 4.6 TB/s for a per-thread id-then-row loop whose two
// dependent round trips cannot overlap as well. Other widths use the per-thread kernel.
// Table rows are read with ordinary loads (a hot Zipf row stays in L2 for its repeats) and the
// output rows are written non-temporally (streamed, no L2 residency for data read once later):
// two-table C3 gather A/B (tools/ab_gather_tables.py, fresh ids per launch) Zipf 21.1 -> 18.0
// us, uniform 24.7 -> 25.0 us against non-temporal loads + ordinary stores.
//
// Backward + update replaces the Embedding IndexedSlices gradient and Keras >= 2.11
// Adagrad.apply_gradients (src/trainer.py:157-163): clip_by_norm over the un-deduplicated
// values, _deduplicate_sparse_grad (segment sum), then the sparse Adagrad row update.
// Deterministic by construction: a stable radix sort of the ids (rocPRIM) gives each table row
// its contributions in input order; one wave per unique row sums them serially and updates
// the row — no float atomics, bit-identical across runs and across data-parallel replicas.
#include "common.hpp"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

namespace rs {

constexpr int kRowsInFlight = 4;

__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ table,
                                                          int64_t num_rows, int64_t q_per_row,
                                                          const int64_t* __restrict__ ids,
                                                          int64_t total_q, float* __restrict__ out,
                                                          int32_t* __restrict__ bad_ids) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const f32x4* t4 = reinterpret_cast<const f32x4*>(table);
  f32x4* o4 = reinterpret_cast<f32x4*>(out);
  for (; i < total_q; i += stride * kRowsInFlight) {
    f32x4 v[kRowsInFlight];
    int64_t idx[kRowsInFlight];
#pragma unroll
    for (int u = 0; u < kRowsInFlight; ++u) {
      idx[u] = i + u * stride;
      v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (idx[u] < total_q) {
        const int64_t row = idx[u] / q_per_row, q = idx[u] - row * q_per_row;
        const int64_t id = ids[row];
        if (id >= 0 && id < num_rows) {
          v[u] = __builtin_nontemporal_load(t4 + id * q_per_row + q);
        } else if (q == 0 && bad_ids) {
          atomicAdd(bad_ids, 1);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kRowsInFlight; ++u)
      if (idx[u] < total_q) o4[idx[u]] = v[u];
  }
}

template <int QPR, int RPW>
__global__ __launch_bounds__(256) void gather_rows_wave_kernel(const float* __restrict__ table, int64_t num_rows,
                                                               const int64_t* __restrict__ ids, int64_t n,
                                                               float* __restrict__ out,
                                                               int32_t* __restrict__ bad_ids) {
  constexpr int RPI = 64 / QPR;  // rows per wave instruction
  constexpr int NI = RPW / RPI;  // row loads in flight per lane
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const f32x4* t4 = reinterpret_cast<const f32x4*>(table);
  f32x4* o4 = reinterpret_cast<f32x4*>(out);
  const int sub = lane / QPR, q = lane % QPR;
  for (int64_t r0 = wave * RPW; r0 < n; r0 += nwaves * RPW) {
    int64_t my_id = -1;
    if (lane < RPW && r0 + lane < n) {
      my_id = ids[r0 + lane];
      if (my_id < 0 || my_id >= num_rows) {
        my_id = -1;
        if (bad_ids) atomicAdd(bad_ids, 1);
      }
    }
    f32x4 v[NI];
    // unconditional loads (an invalid id reads row 0 and is zeroed after): hipcc waits for a load
    // issued under a per-element branch before issuing the next one
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int64_t id = __shfl(my_id, u * RPI + sub);
      v[u] = t4[(id >= 0 ? id : 0) * QPR + q];
      if (id < 0) v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int64_t row = r0 + u * RPI + sub;
      if (row < n) __builtin_nontemporal_store(v[u], o4 + row * QPR + q);
    }
  }
}

template <int QPR>
static void launch_gather_wave(const float* table, int64_t num_rows, const int64_t* ids, int64_t n, float* out,
                               int32_t* bad, hipStream_t st) {
  const int rpw = n >= (1 << 18) ? 64 : 32;
  int64_t blocks = ceil_div(ceil_div(n, rpw), 4);
  if (blocks > 4096) blocks = 4096;
  if (rpw == 64)
    hipLaunchKernelGGL((gather_rows_wave_kernel<QPR, 64>), dim3((unsigned)blocks), dim3(256), 0, st, table,
                       num_rows, ids, n, out, bad);
  else
    hipLaunchKernelGGL((gather_rows_wave_kernel<QPR, 32>), dim3((unsigned)blocks), dim3(256), 0, st, table,
                       num_rows, ids, n, out, bad);
}

// Several tables' gathers in one launch (the user and item lookups of a training step: one
// 135 MB launch at C3 instead of two 68 MB ones, so the launch ramp is paid once). Wave w of
// the concatenated wave space serves table j with wstart[j] <= w < wstart[j + 1].
constexpr int kMaxGatherTables = 8;
struct GatherJobs {
  const float* table[kMaxGatherTables];
  const int64_t* ids[kMaxGatherTables];
  float* out[kMaxGatherTables];
  int64_t num_rows[kMaxGatherTables];
  int64_t n[kMaxGatherTables];
  int64_t wstart[kMaxGatherTables + 1];
  // nullable: position p of table j gathers batch row order[j][p] (rows in ascending-id order from
  // the in-batch id plan, so consecutive lanes read nearby table rows: few TLB pages per wave)
  const int32_t* order[kMaxGatherTables];
  // nullable (distinct rows, rs_embedding_gather_tables_rows_f32): position p gathers the id of batch
  // row rep[j][p] into row p, for p below the device count *count[j] (positions past it are skipped)
  const int32_t* rep[kMaxGatherTables];
  const int64_t* count[kMaxGatherTables];
  // (rs_embedding_gather_tables_ids_f32) a negative id marks a position past the plan's distinct
  // count: not written (instead of a zero row)
  bool skip_neg[kMaxGatherTables];
  int ntables;
};

template <int QPR, int RPW>
__global__ __launch_bounds__(256) void gather_tables_wave_kernel(GatherJobs jobs, int32_t* __restrict__ bad_ids) {
  constexpr int RPI = 64 / QPR;
  constexpr int NI = RPW / RPI;
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int sub = lane / QPR, q = lane % QPR;
  const int64_t wtot = jobs.wstart[jobs.ntables];
  for (int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < wtot; w += nwaves) {
    int j = 0;
#pragma unroll
    for (int k = 1; k < kMaxGatherTables; ++k)
      if (k < jobs.ntables && w >= jobs.wstart[k]) j = k;
    const f32x4* t4 = reinterpret_cast<const f32x4*>(jobs.table[j]);
    f32x4* o4 = reinterpret_cast<f32x4*>(jobs.out[j]);
    int64_t n = jobs.n[j];
    const int64_t num_rows = jobs.num_rows[j];
    if (jobs.count[j]) {
      const int64_t c = *jobs.count[j];
      n = c < n ? (c > 0 ? c : 0) : n;
    }
    const int64_t r0 = (w - jobs.wstart[j]) * RPW;
    if (r0 >= n) continue;  // a wave wholly past the device count: no loads (wave-uniform)
    const int32_t* __restrict__ order = jobs.order[j];
    const int32_t* __restrict__ rep = jobs.rep[j];
    // my_id: the table row, -1 an out-of-range id (a zero row), -2 a position not written
    int64_t my_id = -2, my_row = r0 + lane;
    if (lane < RPW && r0 + lane < n) {
      if (order) my_row = order[r0 + lane];
      my_id = jobs.ids[j][rep ? (int64_t)rep[r0 + lane] : my_row];
      if (my_id < 0 && jobs.skip_neg[j]) {
        my_id = -2;
      } else if (my_id < 0 || my_id >= num_rows) {
        my_id = -1;
        if (bad_ids) atomicAdd(bad_ids, 1);
      }
    }
    // distinct ids: positions past the plan's count are -1 from the count on, so a wave whose first
    // position is one has nothing to gather (wave-uniform exit, no row loads)
    if (jobs.skip_neg[j] && __shfl(my_id, 0) == -2) continue;
    f32x4 v[NI];
#pragma unroll
    for (int u = 0; u < NI; ++u) {  // unconditional loads, as in gather_rows_wave_kernel
      const int64_t id = __shfl(my_id, u * RPI + sub);
      v[u] = t4[(id >= 0 ? id : 0) * QPR + q];
      if (id < 0) v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int64_t pos = r0 + u * RPI + sub;
      const int64_t row = order ? __shfl(my_row, u * RPI + sub) : pos;
      if (pos < n && __shfl(my_id, u * RPI + sub) != -2) __builtin_nontemporal_store(v[u], o4 + row * QPR + q);
    }
  }
}

#ifndef GATHER_IDS_RPW
#define GATHER_IDS_RPW 16  // rows per wave of the distinct-id form: 13.4 -> 12.4 us at C3 Zipf (profiles/r06q_gather_ids_rpw.txt)
#endif
template <int QPR>
static void launch_gather_tables(GatherJobs& jobs, int64_t total_rows, int32_t* bad, hipStream_t st) {
  // 64 rows per wave from 2^17 rows on (the C3 step's 2 x 65,536: Zipf 20 -> 18 us, uniform 26 -> 25 us)
  int rpw = total_rows >= (1 << 17) ? 64 : 32;
  if (jobs.skip_neg[0]) rpw = GATHER_IDS_RPW;
  if (rpw == 16) {
    jobs.wstart[0] = 0;
    for (int j = 0; j < jobs.ntables; ++j) jobs.wstart[j + 1] = jobs.wstart[j] + ceil_div(jobs.n[j], 16);
    int64_t blocks = ceil_div(jobs.wstart[jobs.ntables], 4);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL((gather_tables_wave_kernel<QPR, 16>), dim3((unsigned)blocks), dim3(256), 0, st, jobs, bad);
    return;
  }
  jobs.wstart[0] = 0;
  for (int j = 0; j < jobs.ntables; ++j) jobs.wstart[j + 1] = jobs.wstart[j] + ceil_div(jobs.n[j], rpw);
  int64_t blocks = ceil_div(jobs.wstart[jobs.ntables], 4);
  if (blocks > 4096) blocks = 4096;
  if (rpw == 64)
    hipLaunchKernelGGL((gather_tables_wave_kernel<QPR, 64>), dim3((unsigned)blocks), dim3(256), 0, st, jobs, bad);
  else
    hipLaunchKernelGGL((gather_tables_wave_kernel<QPR, 32>), dim3((unsigned)blocks), dim3(256), 0, st, jobs, bad);
}

// Config-5 feature assembly: x0[b] = [T_0[ids[0][b]] || ... || T_{F-1}[ids[F-1][b]] || dense[b] || 0].
// A thread owns one float4 column c4 of x0 (so its feature f and row offset are fixed) for MG_RPB
// consecutive rows: all MG_RPB row loads are issued before the stores (16 B x MG_RPB in flight per
// thread), 32 lanes cover one 512-B table row (E = 128), no 64-bit divisions per element; table rows
// are read with ordinary loads (hot Zipf rows stay in L2), x0 is written non-temporally.
constexpr int MG_RPB = 8;
__global__ __launch_bounds__(256) void multi_gather_kernel(
    const float* const* __restrict__ tables, const int64_t* __restrict__ nrows, int nfeat, int64_t E,
    const int64_t* __restrict__ ids, int64_t B, const float* __restrict__ dense, int64_t nd,
    float* __restrict__ x0, int64_t ld, int32_t* __restrict__ bad_ids) {
  const int q4 = (int)(ld / 4), e4 = (int)(E / 4), emb4 = nfeat * e4;
  const int c4 = blockIdx.x * 256 + threadIdx.x;
  if (c4 >= q4) return;
  const int64_t b0 = (int64_t)blockIdx.y * MG_RPB;
  f32x4 v[MG_RPB];
  if (c4 < emb4) {
    const int f = c4 / e4, q = c4 - f * e4;
    // the table pointer comes from memory: without the global address space the row loads would be
    // flat loads, which hipcc waits for one at a time
    typedef const __attribute__((address_space(1))) f32x4* gf32x4p;
    const gf32x4p t4 = (gf32x4p)(tables[f]);
    const int64_t nr = nrows[f];
    // all ids first, then all row loads (no atomic between them, so nothing orders the loads), then
    // one count of the invalid ids
    int64_t id[MG_RPB];
    int bad = 0;
    bool ok[MG_RPB];
#pragma unroll
    for (int r = 0; r < MG_RPB; ++r) {
      id[r] = ids[f * B + (b0 + r < B ? b0 + r : B - 1)];
      ok[r] = id[r] >= 0 && id[r] < nr;
      bad += (b0 + r < B && !ok[r]) ? 1 : 0;
    }
    // unconditional loads (an invalid id reads row 0 and is zeroed after): a load under a
    // per-element branch is waited for before the next one is issued
#pragma unroll
    for (int r = 0; r < MG_RPB; ++r) v[r] = t4[(ok[r] ? id[r] : 0) * e4 + q];
#pragma unroll
    for (int r = 0; r < MG_RPB; ++r)
      if (!ok[r]) v[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (bad && q == 0 && bad_ids) atomicAdd(bad_ids, bad);
  } else {
    const int64_t j0 = (int64_t)(c4 - emb4) * 4;
#pragma unroll
    for (int r = 0; r < MG_RPB; ++r) {
      v[r] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (b0 + r < B) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (j0 + k < nd) v[r][k] = dense[(b0 + r) * nd + j0 + k];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < MG_RPB; ++r)
    if (b0 + r < B) __builtin_nontemporal_store(v[r], reinterpret_cast<f32x4*>(x0 + (b0 + r) * ld) + c4);
}

// Sparse update jobs: up to SP_MAXT tables updated by one launch sequence (one sort, one fragment
// pass, one apply pass for all of them). The tables' entries sit in one concatenation: table k owns
// positions [off[k], off[k+1]), its n[k] entries first, then padding up to a multiple of the window
// length (so no window of the fragment pass spans two tables, and each table's windows are the
// ones a single-table update would use). Sort key = (k << kbits) | id, with id = num_rows[k] (the
// sentinel: sorted last within the table, never applied) for invalid ids and for padding. One table
// (nt = 1, no padding) gives exactly the keys, windows and sums of the former single-table path.
constexpr int SP_MAXT = 32;
struct SparseJobs {
  const int64_t* ids[SP_MAXT];
  const float* rows[SP_MAXT];   // gradient rows of table k (row stride ld[k])
  int64_t ld[SP_MAXT];
  int64_t n[SP_MAXT];
  int64_t num_rows[SP_MAXT];
  float* table[SP_MAXT];
  float* accum[SP_MAXT];
  const float* sumsq[SP_MAXT];  // clip norm^2 of table k's raw rows
  int64_t off[SP_MAXT + 1];
  int64_t bstart[SP_MAXT + 1];  // sum-of-squares partial blocks of table k: [bstart[k], bstart[k+1])
  // nullable (all tables or none): table k's positions in ascending id order, equal ids in
  // ascending position, out-of-range ids last — the stable sort's result, supplied by the caller
  // (the in-batch id plan's order entry): the prep pass then writes the sorted pairs and the sort
  // is skipped
  const int32_t* order[SP_MAXT];
  // nullable (all tables or none; with order): the plan's run heads — slot p of table k starts at
  // position hstart[k][p] of the sorted sequence, its id is hdid[k][p] (>= num_rows: the group of
  // out-of-range ids, not applied) and *hcount[k] slots exist — so the apply pass runs one wave
  // slice per run head instead of one wave per sorted position
  const int32_t* hstart[SP_MAXT];
  const int64_t* hdid[SP_MAXT];
  const int64_t* hcount[SP_MAXT];
  int64_t hwstart[SP_MAXT + 1];  // head slices of table k: [hwstart[k], hwstart[k+1])
  int nt, kbits;
};

// grid (blocks of the longest table, nt): block (x, k) keys table k's positions x * 256 + tid
__device__ __forceinline__ float decayed_lr(const int64_t* iteration, float lr0, float decay_rate,
                                            int64_t decay_steps) {
  // tf.keras.optimizers.schedules.ExponentialDecay(staircase=True), evaluated in fp32 as TF does.
  const float step = (float)iteration[0];
  const float p = floorf(step / (float)decay_steps);
  return lr0 * powf(decay_rate, p);
}

// lr_out (nullable): the step's learning rate, read from the step counter here by one thread, for
// the apply pass; with iter_inc (the same counter) that thread then advances it — no other
// workgroup of this grid reads the counter, and the update's later passes read lr_out instead, so
// the increment needs no completion ticket (a ticket in the apply pass held each of its ~32K
// workgroups for an atomic round trip)
__global__ void sparse_prep_kernel(SparseJobs jobs, int64_t* __restrict__ keys, int32_t* __restrict__ vals,
                                   unsigned int* __restrict__ zero, const int64_t* iteration = nullptr,
                                   float lr0 = 0.f, float decay_rate = 1.f, int64_t decay_steps = 1,
                                   float* __restrict__ lr_out = nullptr, int64_t* iter_inc = nullptr) {
  if (zero && blockIdx.x == 0 && blockIdx.y == 0) ticket_zero(zero, threadIdx.x, blockDim.x);  // the norm pass's tickets
  if (lr_out && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    lr_out[0] = decayed_lr(iteration, lr0, decay_rate, decay_steps);
    if (iter_inc) iter_inc[0] += 1;
  }
  const int k = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p = jobs.off[k] + j;
  if (p >= jobs.off[k + 1]) return;
  const int64_t nr = jobs.num_rows[k];
  int64_t id = nr, src = j;
  if (j < jobs.n[k]) {
    if (jobs.order[k]) src = jobs.order[k][j];  // presorted: position j of the sorted sequence
    const int64_t v = jobs.ids[k][src];
    if (v >= 0 && v < nr) id = v;
  }
  keys[p] = ((int64_t)k << jobs.kbits) | id;
  vals[p] = (int32_t)(jobs.off[k] + src);
}


// Deterministic segment sum over the sorted ids in two ordered levels (a Zipf-hot id can own
// thousands of rows: one wave summing them serially took ~5 ms per table at B = 65536).
//   A: fixed windows of kWin sorted positions, one wave each, sum each run fragment inside the
//      window (in position order) into frag[first position of the fragment];
//   B: one wave per run head sums the run's fragments (at the head and at every window start
//      inside the run, in order), then applies the Adagrad row update.
// window length: 64 positions per wave at large n, down to 4 when n is small so the fragment
// pass still spreads over >= ~1024 waves (the same value must be used by both passes)
static int sparse_window(int64_t n) {
  int w = 64;
  while (w > 4 && ceil_div(n, w) < 1024) w >>= 1;
  return w;
}

__device__ __forceinline__ float clip_scale_denom(const float* sumsq, float clipnorm) {
  const float ss = sumsq[0];
  const float l2 = ss > 0.f ? sqrtf(ss) : 0.f;
  return fmaxf(l2, clipnorm);  // tf.clip_by_norm: t * clip_norm / maximum(l2norm, clip_norm)
}

template <int NV>
__global__ __launch_bounds__(256) void sparse_fragment_kernel(const int64_t* __restrict__ skeys,
                                                              const int32_t* __restrict__ perm, SparseJobs jobs,
                                                              int64_t total, int64_t dim, float clipnorm, int kWin,
                                                              float* __restrict__ frag) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kWin;
  if (w0 >= total) return;
  const int cnt = (int)(total - w0 < kWin ? total - w0 : kWin);
  const int64_t my_key = lane < cnt ? skeys[w0 + lane] : -1;
  // the window's table (windows never span two tables)
  const int k = __builtin_amdgcn_readfirstlane((int)(skeys[w0] >> jobs.kbits));
  const float* __restrict__ grad = jobs.rows[k];
  const int64_t grad_ld = jobs.ld[k], nk = jobs.n[k];
  const int64_t my_row = lane < cnt ? (int64_t)perm[w0 + lane] - jobs.off[k] : nk;  // >= nk: padding
  const bool clip = clipnorm > 0.f;
  const float denom = clip ? clip_scale_denom(jobs.sumsq[k], clipnorm) : 1.f;
  float acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = 0.f;
  // rows are loaded 8 positions at a time (independent loads in flight), then summed strictly in
  // position order, so the latency of a window is ~cnt/8 round trips, not cnt (32 at a time: 120
  // VGPRs, half the waves per SIMD, 29.5 -> 31.8 us per C3 step: profiles/r06c_c3_kernel_stats.txt)
  constexpr int LB = 8;
  int head = 0;
  for (int p0 = 0; p0 < cnt; p0 += LB) {
    float g[LB][NV];
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      const int p = p0 + j;
      const int64_t row = __shfl(my_row, p < 64 ? p : 63, 64);
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int64_t d = lane + 64 * v;
        g[j][v] = (p < cnt && d < dim && row < nk) ? grad[row * grad_ld + d] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      const int p = p0 + j;
      if (p >= cnt) continue;  // (no break: the loop stays fully unrolled, g in registers)
      const int64_t key = __shfl(my_key, p, 64);
      const int64_t nkey = __shfl(my_key, p + 1 < 64 ? p + 1 : 63, 64);
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[v] += clip ? (g[j][v] * clipnorm) / denom : g[j][v];
      if (p + 1 == cnt || nkey != key) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const int64_t d = lane + 64 * v;
          if (d < dim) frag[(w0 + head) * dim + d] = acc[v];
          acc[v] = 0.f;
        }
        head = p + 1;
      }
    }
  }
}

// Sum of a key's run: the head position's fragment plus the fragments of the later windows that
// start with the same key (keys are sorted: a prefix), in window order. The run's window count
// comes from ballots over 64 window starts at a time (one per lane), so a hot key's run of hundreds
// of windows (kWin = 4 at small n) costs a few scans, not one round trip per window; the fragments
// are then loaded in branch-free batches of 32 (clamped addresses, a select in the sum) with no
// dependence between batches. Lane l owns the NV contiguous columns d0 .. d0 + NV - 1.
template <int NV>
struct SparseVec {
  typedef float type __attribute__((ext_vector_type(NV)));
};
template <int NV>
__device__ __forceinline__ typename SparseVec<NV>::type run_sum(const float* __restrict__ frag,
                                                                const int64_t* __restrict__ skeys, int64_t n,
                                                                int64_t dim, int kWin, int64_t pos, int64_t key,
                                                                int64_t d0, int lane) {
  typedef typename SparseVec<NV>::type fv;
  auto ld = [&](const float* base) -> fv { return *reinterpret_cast<const fv*>(base + d0); };
  fv gs = ld(frag + pos * dim);
  const int64_t q0 = (pos / kWin + 1) * kWin;  // start of the next window
  int64_t nw = 0;
  for (int64_t qs = q0;; qs += 64 * (int64_t)kWin) {
    const int64_t qq = qs + (int64_t)lane * kWin;
    const bool mt = qq < n && skeys[qq] == key;
    const uint64_t miss = __ballot(!mt);
    const int lead = miss ? __ffsll((long long)miss) - 1 : 64;
    nw += lead;
    if (lead < 64) break;
  }
  constexpr int FB = 32;
  for (int64_t w0 = 0; w0 < nw; w0 += FB) {
    fv f[FB];
#pragma unroll
    for (int j = 0; j < FB; ++j) f[j] = ld(frag + (q0 + (w0 + j < nw ? w0 + j : nw - 1) * kWin) * dim);
    const fv zero = {};
#pragma unroll
    for (int j = 0; j < FB; ++j) gs += w0 + j < nw ? f[j] : zero;  // a select, no branch
  }
  return gs;
}

// The Adagrad update of one element (shared by the apply passes: the same arithmetic)
struct AdagradElem {
  float t, a;
};
__device__ __forceinline__ AdagradElem adagrad_row_elem(float tv, float av, float g, float lr, float eps) {
  AdagradElem r;
  r.a = av + g * g;
  r.t = tv - lr * g / sqrtf(r.a + eps);
  return r;
}

// One wave per sorted position; the wave at the head of a key's run applies the run's update
// (run_sum) to its table's row, the table and accumulator rows and the step counter loaded beside
// the run's loads.
template <int NV>
__device__ __forceinline__ void sparse_apply_pos(
    const SparseJobs& jobs, int64_t dim, const int64_t* __restrict__ skeys, const float* __restrict__ frag,
    int64_t total, const float* __restrict__ lr_in, float eps, int kWin) {
  typedef typename SparseVec<NV>::type fv;
  const int lane = threadIdx.x & 63;
  const int64_t pos = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pos >= total) return;
  const int64_t key = skeys[pos];
  const int64_t prev = pos > 0 ? skeys[pos - 1] : -1;
  if (prev == key) return;
  const int k = __builtin_amdgcn_readfirstlane((int)(key >> jobs.kbits));
  const int64_t id = key & (((int64_t)1 << jobs.kbits) - 1);
  if (id >= jobs.num_rows[k]) return;
  float* __restrict__ table = jobs.table[k];
  float* __restrict__ accum = jobs.accum[k];
  // the lane's columns (lanes past dim read the last NV columns and store nothing)
  const int64_t d0 = (int64_t)NV * lane < dim ? (int64_t)NV * lane : dim - NV;
  const bool own = (int64_t)NV * lane < dim;
  const fv tv = *reinterpret_cast<const fv*>(table + id * dim + d0);
  const fv av = *reinterpret_cast<const fv*>(accum + id * dim + d0);
  const float lr = lr_in[0];
  const fv gs = run_sum<NV>(frag, skeys, total, dim, kWin, pos, key, d0, lane);
  if (own) {
    fv a, t;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const AdagradElem e = adagrad_row_elem(tv[v], av[v], gs[v], lr, eps);
      a[v] = e.a;
      t[v] = e.t;
    }
    *reinterpret_cast<fv*>(accum + id * dim + d0) = a;
    *reinterpret_cast<fv*>(table + id * dim + d0) = t;
  }
}

// (the step's learning rate from lr_in, formed by the prep pass, which also advanced the step
// counter when asked)
template <int NV>
__global__ __launch_bounds__(256, 2) void sparse_apply_kernel(
    SparseJobs jobs, int64_t dim, const int64_t* __restrict__ skeys, const float* __restrict__ frag, int64_t total,
    const float* __restrict__ lr_in, float eps, int kWin) {
  sparse_apply_pos<NV>(jobs, dim, skeys, frag, total, lr_in, eps, kWin);
}

// The apply pass over the plan's run heads (SparseJobs hstart / hdid / hcount): LPH lanes own one
// head (4 contiguous columns each: LPH = dim / 4), 64 / LPH heads per wave. A head's run is
// [start, next start) (the table's entry count after its last slot); its sum is run_sum's — the
// head's fragment, then the fragments at the window starts inside the run in window order, loaded in
// branch-free batches of 32 with a select — and its Adagrad row update the same arithmetic
// (adagrad_row_elem), so every row is bitwise sparse_apply_kernel's. Two dependent load levels per
// head (start and id, then the rows and fragments) instead of the per-position wave's key, previous
// key, ballot scan and fragments, and one slice per distinct id instead of a wave per position.
// The sum of a run [pos, end) of sorted positions from its fragments: the head's fragment, then
// the fragments at the window starts inside the run in window order (8 loads in flight). run_sum's
// batches of 32 also add +0 for the clamped slots of a partial last batch, which only turns a -0 sum
// into +0: one +0 add here, so the result is bitwise run_sum's.
__device__ __forceinline__ SparseVec<4>::type heads_run_sum(const float* __restrict__ frag, int64_t dim, int64_t d0,
                                                            int64_t pos, int64_t end, int kWin) {
  typedef SparseVec<4>::type fv;
  auto ld = [&](int64_t q) -> fv { return *reinterpret_cast<const fv*>(frag + q * dim + d0); };
  fv gs = ld(pos);
  const int64_t q0 = (pos / kWin + 1) * kWin;   // the first window start after the head
  const int64_t nw = end > q0 ? (end - q0 + kWin - 1) / kWin : 0;
  constexpr int FB = 8;
  const fv zero = {};
  for (int64_t w0 = 0; w0 < nw; w0 += FB) {
    fv f[FB];
#pragma unroll
    for (int j = 0; j < FB; ++j) f[j] = ld(q0 + (w0 + j < nw ? w0 + j : nw - 1) * kWin);
#pragma unroll
    for (int j = 0; j < FB; ++j)
      if (w0 + j < nw) gs += f[j];
  }
  if (nw % 32) gs += zero;
  return gs;
}

template <int LPH>
__global__ __launch_bounds__(256) void sparse_apply_heads_kernel(SparseJobs jobs, int64_t dim,
                                                                 const float* __restrict__ frag,
                                                                 const float* __restrict__ lr_in, float eps,
                                                                 int kWin) {
  constexpr int HPW = 64 / LPH;
  const int lane = threadIdx.x & 63, hl = lane / LPH, c4 = lane % LPH;
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (w >= jobs.hwstart[jobs.nt]) return;
  int k = 0;
  for (int q = 1; q < jobs.nt; ++q)
    if (w >= jobs.hwstart[q]) k = q;
  const int64_t nslots = *jobs.hcount[k];
  const int64_t p = (w - jobs.hwstart[k]) * HPW + hl;
  if (p >= nslots) return;  // (whole head slices: every lane of a slice leaves together)
  const int64_t nk = jobs.n[k];
  const int64_t s0 = jobs.hstart[k][p];
  const int64_t s1 = p + 1 < nslots ? (int64_t)jobs.hstart[k][p + 1] : nk;
  const int64_t id = jobs.hdid[k][p];
  if (id < 0 || id >= jobs.num_rows[k]) return;
  typedef typename SparseVec<4>::type fv;
  const int64_t d0 = 4 * (int64_t)c4;
  float* __restrict__ table = jobs.table[k];
  float* __restrict__ accum = jobs.accum[k];
  const fv tv = *reinterpret_cast<const fv*>(table + id * dim + d0);
  const fv av = *reinterpret_cast<const fv*>(accum + id * dim + d0);
  const float lr = lr_in[0];
  const fv gs = heads_run_sum(frag, dim, d0, jobs.off[k] + s0, jobs.off[k] + s1, kWin);
  fv a, t;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const AdagradElem e = adagrad_row_elem(tv[v], av[v], gs[v], lr, eps);
    a[v] = e.a;
    t[v] = e.t;
  }
  *reinterpret_cast<fv*>(accum + id * dim + d0) = a;
  *reinterpret_cast<fv*>(table + id * dim + d0) = t;
}

// Per-table clip norms^2 of the raw rows in two launches for all tables, each table's partials and
// tree exactly those of launch_sumsq_2d (sumsq_blocks(n dim) blocks striding over the table's
// elements, then final_sum_kernel's tree): grid (most blocks of a table, nt), then one workgroup
// per table.
__device__ void sparse_sumsq_final_block(const SparseJobs& jobs, const double* __restrict__ part,
                                         float* __restrict__ out, int k, double* red);

// with `done` (zeroed by sparse_prep_kernel) the last workgroup to finish also runs the final of
// every table (one 256-thread tree per table, in table order) instead of another launch
__global__ __launch_bounds__(256) void sparse_sumsq_partial_kernel(SparseJobs jobs, int64_t dim,
                                                                   double* __restrict__ part,
                                                                   unsigned int* __restrict__ done = nullptr,
                                                                   float* __restrict__ out = nullptr) {
  __shared__ double red[256];
  const int k = blockIdx.y;
  const int64_t nb = jobs.bstart[k + 1] - jobs.bstart[k];
  if ((int64_t)blockIdx.x < nb) {
    const float* __restrict__ x = jobs.rows[k];
    const int64_t ld = jobs.ld[k], n = jobs.n[k] * dim;
    double acc = 0.0;
    // the element order of the 2-D form in every case; the row / column split only for strided
    // rows, and in 32 bits when it fits (a 64-bit division per element made this pass VALU-bound:
    // 31.6 us for C3's 2 x 8.4 M elements)
    const bool dense = ld == dim, narrow = n <= 0xffffffffLL;
    auto at = [&](int64_t i) -> float {
      if (dense) return x[i];
      if (narrow) {
        const uint32_t r = (uint32_t)i / (uint32_t)dim;
        return x[(int64_t)r * ld + ((uint32_t)i - r * (uint32_t)dim)];
      }
      const int64_t r = i / dim;
      return x[r * ld + (i - r * dim)];
    };
    // eight elements' loads in flight before they are accumulated (in the same order; 32 in flight
    // measured 24.2 -> 25.7 us per C3 step, round 6)
    const int64_t step = nb * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 7 * step < n; i += 8 * step) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = at(i + u * step);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += (double)v[u] * (double)v[u];
    }
    for (; i < n; i += step) {
      const float v = at(i);
      acc += (double)v * (double)v;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      if (done) ticket_publish(part + jobs.bstart[k] + blockIdx.x, red[0]);
      else part[jobs.bstart[k] + blockIdx.x] = red[0];
    }
  }
  if (!done) return;
  // the last workgroup reads the published partials agent-coherently (common.hpp tickets)
  if (!ticket_last(done, (int64_t)blockIdx.y * gridDim.x + blockIdx.x, (int64_t)gridDim.x * gridDim.y)) return;
  for (int t = 0; t < jobs.nt; ++t) {
    sparse_sumsq_final_block(jobs, part, out, t, red);
    __syncthreads();
  }
}

__device__ void sparse_sumsq_final_block(const SparseJobs& jobs, const double* __restrict__ part,
                                         float* __restrict__ out, int k, double* red) {
  const int64_t b0 = jobs.bstart[k], np = jobs.bstart[k + 1] - b0;
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < np; i += 256) acc += ticket_collect(part + b0 + i);
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[k] = (float)red[0];
}

// Local deduplication for the data-parallel exchange: the run of each valid id (sorted keys) is
// summed from its window fragments (the same ordered sums as sparse_apply_kernel) and written to
// output slot slots[pos] (exclusive scan of the run-head flags): unique ids ascending.
__global__ void dedupe_flags_kernel(const int64_t* __restrict__ skeys, int64_t n, int64_t num_rows,
                                    int32_t* __restrict__ flags) {
  const int64_t pos = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (pos >= n) return;
  const int64_t key = skeys[pos];
  flags[pos] = (key < num_rows && (pos == 0 || skeys[pos - 1] != key)) ? 1 : 0;
}

template <int NV>
__global__ __launch_bounds__(256, 2) void dedupe_apply_kernel(
    const int64_t* __restrict__ skeys, const float* __restrict__ frag, int64_t n, int64_t dim, int64_t num_rows,
    int kWin, const int32_t* __restrict__ slots, int64_t* __restrict__ out_ids, float* __restrict__ out_rows,
    int64_t* __restrict__ out_count) {
  typedef typename SparseVec<NV>::type fv;
  const int lane = threadIdx.x & 63;
  const int64_t pos = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pos >= n) return;
  const int64_t key = skeys[pos];
  const int64_t prev = pos > 0 ? skeys[pos - 1] : -1;
  if (pos == n - 1 && lane == 0) {
    const bool head = key < num_rows && (pos == 0 || prev != key);
    out_count[0] = (int64_t)slots[pos] + (head ? 1 : 0);
  }
  if (key >= num_rows || prev == key) return;
  const int64_t d0 = (int64_t)NV * lane < dim ? (int64_t)NV * lane : dim - NV;
  const int64_t slot = slots[pos];
  const fv gs = run_sum<NV>(frag, skeys, n, dim, kWin, pos, key, d0, lane);
  if (lane == 0) out_ids[slot] = key;
  if ((int64_t)NV * lane < dim) *reinterpret_cast<fv*>(out_rows + slot * dim + d0) = gs;
}

// The local deduplication over an id plan's run heads (rs_sparse_dedupe_planned_f32): slot p of the
// plan (ascending ids) -> out_ids[p] = its id, out_rows[p] = its run's sum (heads_run_sum: bitwise
// dedupe_apply_kernel's); the group of out-of-range ids is the plan's last slot and is dropped.
template <int LPH>
__global__ __launch_bounds__(256) void dedupe_heads_kernel(const int32_t* __restrict__ hstart,
                                                           const int64_t* __restrict__ hdid,
                                                           const int64_t* __restrict__ hcount, int64_t n,
                                                           int64_t dim, int64_t num_rows, int kWin,
                                                           const float* __restrict__ frag,
                                                           int64_t* __restrict__ out_ids, float* __restrict__ out_rows,
                                                           int64_t* __restrict__ out_count) {
  constexpr int HPW = 64 / LPH;
  const int lane = threadIdx.x & 63, hl = lane / LPH, c4 = lane % LPH;
  const int64_t p = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * HPW + hl;
  const int64_t nslots = *hcount;
  if (p == 0 && lane == 0) out_count[0] = nslots - (nslots > 0 && hdid[nslots - 1] >= num_rows ? 1 : 0);
  if (p >= nslots) return;
  const int64_t id = hdid[p];
  if (id < 0 || id >= num_rows) return;
  const int64_t s0 = hstart[p], s1 = p + 1 < nslots ? (int64_t)hstart[p + 1] : n;
  const int64_t d0 = 4 * (int64_t)c4;
  const SparseVec<4>::type gs = heads_run_sum(frag, dim, d0, s0, s1, kWin);
  if (c4 == 0) out_ids[p] = id;
  *reinterpret_cast<SparseVec<4>::type*>(out_rows + p * dim + d0) = gs;
}

__global__ void sumsq_to_f32_kernel(const float* __restrict__ in, float* __restrict__ out) { out[0] = in[0]; }

// One-workgroup stable LSD radix sort of up to LDS_SORT_MAX (key, value) pairs whose keys are
// below 2^32 (the sparse Adagrad's (table, id) keys at C2-sized batches): 8-bit digits, every pass
// in LDS, one launch instead of rocprim's block sort + merge passes (6 launches, ~29 us at 8192
// pairs). Wave w ranks its 512 items in index order (ballot peer groups), digit-major / wave-minor
// offsets: equal keys keep their input order, so the result is the one any stable sort gives.
constexpr int LDS_SORT_MAX = 8192;
// Segments (seg, optional): workgroup b sorts positions [seg->off[b], seg->off[b + 1]) on its own —
// the tables of the sparse update, whose keys carry the table index above the id bits, so the
// stable sort of the whole sequence is the concatenation of the tables' stable sorts by id bits.
struct LdsSortSegs {
  int64_t off[SP_MAXT + 1];
};
__global__ __launch_bounds__(1024) void lds_sort_pairs_kernel(const int64_t* __restrict__ kin,
                                                              const int32_t* __restrict__ vin,
                                                              int64_t* __restrict__ kout, int32_t* __restrict__ vout,
                                                              int n, int end_bit, LdsSortSegs seg = {}) {
  __shared__ uint32_t kbuf[2][LDS_SORT_MAX];
  __shared__ int32_t vbuf[2][LDS_SORT_MAX];
  __shared__ uint32_t hist[256 * 16];  // [digit][wave]: counts, then running offsets
  __shared__ uint32_t wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (gridDim.x > 1) {
    const int64_t b0 = seg.off[blockIdx.x];
    kin += b0;
    vin += b0;
    kout += b0;
    vout += b0;
    n = (int)(seg.off[blockIdx.x + 1] - b0);
  }
  for (int i = tid; i < n; i += 1024) {
    kbuf[0][i] = (uint32_t)kin[i];
    vbuf[0][i] = vin[i];
  }
  int cur = 0;
  for (int bit = 0; bit < end_bit; bit += 8) {
    for (int d = tid; d < 256 * 16; d += 1024) hist[d] = 0u;
    __syncthreads();
    const uint32_t* ks = kbuf[cur];
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      const int i = wave * 512 + st * 64 + lane;
      if (i < n) atomicAdd(&hist[((ks[i] >> bit) & 255u) * 16 + wave], 1u);
    }
    __syncthreads();
    // exclusive scan of the 4096 counts in digit-major order: 4 per thread, then across threads
    uint32_t c[4], loc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c[j] = hist[4 * tid + j];
      loc += c[j];
    }
    uint32_t inc = loc;  // inclusive scan over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t wofs = 0;
    for (int w = 0; w < wave; ++w) wofs += wsum[w];
    uint32_t run = wofs + inc - loc;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      hist[4 * tid + j] = run;
      run += c[j];
    }
    __syncthreads();
    uint32_t* kd = kbuf[cur ^ 1];
    int32_t* vd = vbuf[cur ^ 1];
    const int32_t* vs = vbuf[cur];
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      const int i = wave * 512 + st * 64 + lane;
      const bool live = i < n;
      const uint32_t key = live ? ks[i] : 0u;
      const uint32_t dg = (key >> bit) & 255u;
      uint64_t peers = __ballot(live);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const uint64_t bb = __ballot((dg >> b) & 1u);
        peers &= ((dg >> b) & 1u) ? bb : ~bb;
      }
      const int rank = __popcll(peers & ((1ull << lane) - 1ull));
      const uint32_t base = hist[dg * 16 + wave];
      if (live) {
        kd[base + rank] = key;
        vd[base + rank] = vs[i];
      }
      // the group's last lane advances the wave's running offset (read above by every lane first:
      // one wave's LDS operations complete in order)
      if (live && (peers >> lane) == 1ull) hist[dg * 16 + wave] = base + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    cur ^= 1;
  }
  for (int i = tid; i < n; i += 1024) {
    kout[i] = (int64_t)kbuf[cur][i];
    vout[i] = vbuf[cur][i];
  }
}

// The rocprim sort of the sparse update's keys. Its temp-size query (temp == nullptr) and the sort
// itself go through this one function (same config; the query takes the widest bit range, which
// bounds every narrower one's temp), so they cannot diverge.
static hipError_t rocprim_sort_i64(void* temp, size_t& bytes, const int64_t* kin, int64_t* kout, const int32_t* vin,
                                   int32_t* vout, int64_t n, int end_bit, hipStream_t st) {
  return rocprim::radix_sort_pairs(temp, bytes, kin, kout, vin, vout, (unsigned)(n > 0 ? n : 1), 0u,
                                   (unsigned)end_bit, st);
}

// (key, value) pairs sorted by key, stable: the one-workgroup LDS sort when it fits, else rocprim
// (RS_SORT_LDS=0 forces rocprim: read per call, so a test can compare the two in one process)
static hipError_t sort_pairs_i64(void* temp, size_t tb, const int64_t* kin, int64_t* kout, const int32_t* vin,
                                 int32_t* vout, int64_t n, int end_bit, hipStream_t st) {
  const char* env = exp_env("RS_SORT_LDS");
  if (n <= LDS_SORT_MAX && end_bit <= 32 && !(env && env[0] == '0')) {
    hipLaunchKernelGGL(lds_sort_pairs_kernel, dim3(1), dim3(1024), 0, st, kin, vin, kout, vout, (int)n, end_bit);
    return hipGetLastError();
  }
  return rocprim_sort_i64(temp, tb, kin, kout, vin, vout, n, end_bit, st);
}

static int sort_temp_bytes(int64_t n, size_t* bytes) {
  *bytes = 0;
  hipError_t e = rocprim_sort_i64(nullptr, *bytes, nullptr, nullptr, nullptr, nullptr, n, 64, (hipStream_t)0);
  return e == hipSuccess ? RS_OK : RS_ERR_HIP;
}

static int key_bits(int64_t num_rows) {
  int b = 1;
  while (b < 63 && ((int64_t)1 << b) <= num_rows) ++b;  // must represent num_rows (sentinel)
  return b;
}

// Positions of the tables in the padded concatenation (SparseJobs) and the window length: the
// window of the shortest non-empty table (the single-table choice when all tables are equal),
// every table but the last padded to a multiple of it. Returns the total position count.
static int64_t sparse_layout(int nt, const int64_t* n, int* kwin, int64_t* off) {
  int64_t nmin = -1;
  for (int k = 0; k < nt; ++k)
    if (n[k] > 0 && (nmin < 0 || n[k] < nmin)) nmin = n[k];
  const int w = sparse_window(nmin > 0 ? nmin : 1);
  if (kwin) *kwin = w;
  int64_t o = 0;
  for (int k = 0; k < nt; ++k) {
    if (off) off[k] = o;
    o += k + 1 < nt ? ceil_div(n[k], w) * w : n[k];
  }
  if (off) off[nt] = o;
  return o;
}

static size_t sparse_ws_bytes(int nt, const int64_t* n, int64_t dim) {
  const int64_t total = sparse_layout(nt, n, nullptr, nullptr);
  size_t tb = 0;
  if (sort_temp_bytes(total, &tb) != RS_OK) return 0;
  int64_t nb = 0;
  for (int k = 0; k < nt; ++k) nb += sumsq_blocks(n[k] * dim);
  Carve c(nullptr, 0);
  c.take<int64_t>(total);
  c.take<int32_t>(total);
  c.take<int64_t>(total);
  c.take<int32_t>(total);
  c.take<double>(nb > 0 ? nb : 1);
  c.take<float>(nt > 4 ? nt : 4);
  c.take<float>((size_t)total * dim);
  c.take<char>(tb);
  c.take<unsigned int>(TICKET_WORDS);
  c.take<float>(4);
  return c.off + 256;
}

// the update of the tables in jobs (ids, rows, ld, n, num_rows, table, accum filled; sumsq[k] filled
// when the caller supplies the clip norms^2, else sumsq_ext == false and they are computed here)
static int sparse_run(SparseJobs& jobs, int64_t dim, const int64_t* iteration, float lr0, float decay_rate,
                      int64_t decay_steps, float clipnorm, float epsilon, bool sumsq_ext, void* workspace,
                      size_t workspace_bytes, hipStream_t st, int64_t* iter_inc = nullptr) {
  const int nt = jobs.nt;
  int kWin = 4;
  const int64_t total = sparse_layout(nt, jobs.n, &kWin, jobs.off);
  if (total == 0) return RS_OK;
  int64_t nr_max = 1, nblk = 1;
  jobs.bstart[0] = 0;
  for (int k = 0; k < nt; ++k) {
    nr_max = jobs.num_rows[k] > nr_max ? jobs.num_rows[k] : nr_max;
    jobs.bstart[k + 1] = jobs.bstart[k] + sumsq_blocks(jobs.n[k] * dim);
    const int64_t len = jobs.off[k + 1] - jobs.off[k];
    nblk = ceil_div(len, 256) > nblk ? ceil_div(len, 256) : nblk;
  }
  jobs.kbits = key_bits(nr_max);
  const int end_bit = jobs.kbits + (nt > 1 ? key_bits(nt - 1) : 0);
  const size_t need = sparse_ws_bytes(nt, jobs.n, dim);
  if (!workspace || workspace_bytes < need || need == 0) {
    set_error("rs_sparse_adagrad: workspace too small (%zu < %zu)", workspace_bytes, need);
    return RS_ERR_WORKSPACE;
  }
  size_t tb = 0;
  if (sort_temp_bytes(total, &tb) != RS_OK) {
    set_error("rs_sparse_adagrad: rocprim temp query failed");
    return RS_ERR_HIP;
  }
  Carve c(workspace, workspace_bytes);
  int64_t* keys_in = c.take<int64_t>(total);
  int32_t* vals_in = c.take<int32_t>(total);
  int64_t* keys_out = c.take<int64_t>(total);
  int32_t* vals_out = c.take<int32_t>(total);
  double* part = c.take<double>(jobs.bstart[nt] > 0 ? jobs.bstart[nt] : 1);
  float* ssq = c.take<float>(nt > 4 ? nt : 4);
  float* frag = c.take<float>((size_t)total * dim);
  char* temp = c.take<char>(tb);
  unsigned int* done = c.take<unsigned int>(TICKET_WORDS);
  float* lr = c.take<float>(4);

  const bool norms = clipnorm > 0.f && !sumsq_ext;
  const bool presorted = jobs.order[0] != nullptr;
  // several tables that each fit one workgroup's LDS sort: one workgroup per table, sorting by the
  // id bits (the table bits above them are constant per table) — bitwise the one-sequence sort
  bool segmented = !presorted && nt > 1 && jobs.kbits + key_bits(nt - 1) <= 32;
  for (int k = 0; k < nt && segmented; ++k) segmented = jobs.off[k + 1] - jobs.off[k] <= LDS_SORT_MAX;
  {
    const char* env = exp_env("RS_SORT_LDS");
    if (env && env[0] == '0') segmented = false;
  }
  hipLaunchKernelGGL(sparse_prep_kernel, dim3((unsigned)nblk, (unsigned)nt), dim3(256), 0, st, jobs,
                     presorted ? keys_out : keys_in, presorted ? vals_out : vals_in, norms ? done : nullptr, iteration,
                     lr0, decay_rate, decay_steps, lr, iter_inc);
  int rc = check_launch("sparse_prep");
  if (rc) return rc;
  if (segmented) {
    LdsSortSegs seg{};
    for (int k = 0; k <= nt; ++k) seg.off[k] = jobs.off[k];
    hipLaunchKernelGGL(lds_sort_pairs_kernel, dim3((unsigned)nt), dim3(1024), 0, st, keys_in, vals_in, keys_out,
                       vals_out, 0, jobs.kbits, seg);
    rc = check_launch("lds_sort_segments");
    if (rc) return rc;
  } else if (!presorted) {
    hipError_t e = sort_pairs_i64(temp, tb, keys_in, keys_out, vals_in, vals_out, total, end_bit, st);
    if (e != hipSuccess) {
      set_error("rs_sparse_adagrad: radix sort failed: %s", hipGetErrorString(e));
      return RS_ERR_HIP;
    }
  }
  if (clipnorm > 0.f && !sumsq_ext) {
    int64_t bmax = 1;
    for (int k = 0; k < nt; ++k) {
      const int64_t b = jobs.bstart[k + 1] - jobs.bstart[k];
      bmax = b > bmax ? b : bmax;
    }
    // the partials' last workgroup forms every table's norm^2 (the ticket zeroed by the prep pass)
    hipLaunchKernelGGL(sparse_sumsq_partial_kernel, dim3((unsigned)bmax, (unsigned)nt), dim3(256), 0, st, jobs, dim,
                       part, done, ssq);
    rc = check_launch("sparse_sumsq_partial");
    if (rc) return rc;
    for (int k = 0; k < nt; ++k) jobs.sumsq[k] = ssq + k;
  }
  const int nv = (int)ceil_div(dim, 64);
  const unsigned gw = (unsigned)ceil_div(ceil_div(total, kWin), 4);
  const unsigned ga = (unsigned)ceil_div(total, 4);
  // the plan's run heads: one LPH-lane slice per head (dim 32 .. 256)
  const int lph = (int)(dim / 4);
  const bool heads = jobs.hstart[0] != nullptr && presorted && dim % 4 == 0 &&
                     (lph == 8 || lph == 16 || lph == 32 || lph == 64);
  if (heads) {
    jobs.hwstart[0] = 0;
    for (int k = 0; k < nt; ++k) jobs.hwstart[k + 1] = jobs.hwstart[k] + ceil_div(jobs.n[k], 64 / lph);
  }
  const unsigned gh = (unsigned)ceil_div(jobs.hwstart[nt], 4);
#define RS_SPARSE(NV)                                                                                       \
  hipLaunchKernelGGL((sparse_fragment_kernel<NV>), dim3(gw), dim3(256), 0, st, keys_out, vals_out, jobs, total, \
                     dim, clipnorm, kWin, frag);                                                            \
  rc = check_launch("sparse_fragment");                                                                    \
  if (rc) return rc;                                                                                       \
  if (heads) {                                                                                             \
    if (lph == 8) hipLaunchKernelGGL((sparse_apply_heads_kernel<8>), dim3(gh), dim3(256), 0, st, jobs, dim, frag, lr, epsilon, kWin); \
    else if (lph == 16) hipLaunchKernelGGL((sparse_apply_heads_kernel<16>), dim3(gh), dim3(256), 0, st, jobs, dim, frag, lr, epsilon, kWin); \
    else if (lph == 32) hipLaunchKernelGGL((sparse_apply_heads_kernel<32>), dim3(gh), dim3(256), 0, st, jobs, dim, frag, lr, epsilon, kWin); \
    else hipLaunchKernelGGL((sparse_apply_heads_kernel<64>), dim3(gh), dim3(256), 0, st, jobs, dim, frag, lr, epsilon, kWin); \
  } else {                                                                                                 \
    hipLaunchKernelGGL((sparse_apply_kernel<NV>), dim3(ga), dim3(256), 0, st, jobs, dim, keys_out, frag, total, \
                       lr, epsilon, kWin);                                                                 \
  }
  if (nv <= 1) { RS_SPARSE(1) }
  else if (nv <= 2) { RS_SPARSE(2) }
  else if (nv <= 4) { RS_SPARSE(4) }
  else {
    set_error("rs_sparse_adagrad: dim must be <= 256");
    return RS_ERR_UNSUPPORTED;
  }
#undef RS_SPARSE
  return check_launch("sparse_apply");
}

}  // namespace rs

using namespace rs;

extern "C" {

int rs_embedding_gather_f32(const float* table, int64_t num_rows, int64_t dim,
                            const int64_t* ids, int64_t n, float* out, int32_t* bad_ids,
                            rs_stream_t stream) {
  RS_REQUIRE(num_rows > 0 && dim > 0 && n >= 0, "rs_embedding_gather_f32: bad sizes");
  RS_REQUIRE(dim % 4 == 0, "rs_embedding_gather_f32: dim must be a multiple of 4");
  RS_REQUIRE(table && (n == 0 || (ids && out)), "rs_embedding_gather_f32: null pointer");
  if (n == 0) return RS_OK;
  RS_REQUIRE(aligned16(table) && aligned16(out), "rs_embedding_gather_f32: 16-byte alignment");
  const int64_t qpr = dim / 4, total = n * qpr;
  hipStream_t st = as_stream(stream);
  if (qpr == 32 || qpr == 16 || qpr == 8) {
    if (qpr == 32) launch_gather_wave<32>(table, num_rows, ids, n, out, bad_ids, st);
    else if (qpr == 16) launch_gather_wave<16>(table, num_rows, ids, n, out, bad_ids, st);
    else launch_gather_wave<8>(table, num_rows, ids, n, out, bad_ids, st);
    return check_launch("embedding_gather");
  }
  int64_t blocks = ceil_div(total, 256 * 2);
  if (blocks > 256 * 16) blocks = 256 * 16;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     table, num_rows, qpr, ids, total, out, bad_ids);
  return check_launch("embedding_gather");
}

static int gather_tables(int ntables, const float* const* tables, const int64_t* num_rows,
                         const int64_t* const* ids, const int32_t* const* orders, const int64_t* n,
                         float* const* outs, int64_t dim, int32_t* bad_ids, rs_stream_t stream,
                         const int32_t* const* reps = nullptr, const int64_t* const* counts = nullptr,
                         bool skip_neg = false) {
  RS_REQUIRE(ntables >= 0 && ntables <= kMaxGatherTables, "rs_embedding_gather_tables_f32: 0..8 tables");
  RS_REQUIRE(dim > 0 && dim % 4 == 0, "rs_embedding_gather_tables_f32: dim must be a positive multiple of 4");
  RS_REQUIRE(ntables == 0 || (tables && num_rows && ids && n && outs), "rs_embedding_gather_tables_f32: null array");
  const int64_t qpr = dim / 4;
  GatherJobs jobs{};
  jobs.ntables = 0;
  int64_t total = 0;
  for (int j = 0; j < ntables; ++j) {
    RS_REQUIRE(num_rows[j] > 0 && n[j] >= 0, "rs_embedding_gather_tables_f32: bad sizes (table %d)", j);
    if (n[j] == 0) continue;
    RS_REQUIRE(tables[j] && ids[j] && outs[j], "rs_embedding_gather_tables_f32: null pointer (table %d)", j);
    RS_REQUIRE(aligned16(tables[j]) && aligned16(outs[j]), "rs_embedding_gather_tables_f32: 16-byte alignment");
    const int k = jobs.ntables++;
    jobs.table[k] = tables[j];
    jobs.ids[k] = ids[j];
    jobs.out[k] = outs[j];
    jobs.num_rows[k] = num_rows[j];
    jobs.n[k] = n[j];
    jobs.order[k] = orders ? orders[j] : nullptr;
    jobs.rep[k] = reps ? reps[j] : nullptr;
    jobs.count[k] = counts ? counts[j] : nullptr;
    jobs.skip_neg[k] = skip_neg;
    total += n[j];
  }
  if (total == 0) return RS_OK;
  hipStream_t st = as_stream(stream);
  if (qpr == 32) launch_gather_tables<32>(jobs, total, bad_ids, st);
  else if (qpr == 16) launch_gather_tables<16>(jobs, total, bad_ids, st);
  else if (qpr == 8) launch_gather_tables<8>(jobs, total, bad_ids, st);
  else {
    RS_REQUIRE(!reps && !counts, "rs_embedding_gather_tables_rows_f32: dim must be 32, 64 or 128");
    for (int j = 0; j < jobs.ntables; ++j) {
      // (an order only changes the order of the row copies, not their result)
      const int rc = rs_embedding_gather_f32(jobs.table[j], jobs.num_rows[j], dim, jobs.ids[j], jobs.n[j],
                                             jobs.out[j], bad_ids, stream);
      if (rc) return rc;
    }
    return RS_OK;
  }
  return check_launch("embedding_gather_tables");
}

int rs_embedding_gather_tables_f32(int ntables, const float* const* tables, const int64_t* num_rows,
                                   const int64_t* const* ids, const int64_t* n, float* const* outs,
                                   int64_t dim, int32_t* bad_ids, rs_stream_t stream) {
  return gather_tables(ntables, tables, num_rows, ids, nullptr, n, outs, dim, bad_ids, stream);
}

int rs_embedding_gather_tables_ordered_f32(int ntables, const float* const* tables, const int64_t* num_rows,
                                           const int64_t* const* ids, const int32_t* const* orders,
                                           const int64_t* n, float* const* outs, int64_t dim, int32_t* bad_ids,
                                           rs_stream_t stream) {
  RS_REQUIRE(orders, "rs_embedding_gather_tables_ordered_f32: null orders");
  return gather_tables(ntables, tables, num_rows, ids, orders, n, outs, dim, bad_ids, stream);
}

int rs_embedding_gather_tables_rows_f32(int ntables, const float* const* tables, const int64_t* num_rows,
                                        const int64_t* const* ids, const int32_t* const* reps,
                                        const int64_t* const* counts, const int64_t* n, float* const* outs,
                                        int64_t dim, int32_t* bad_ids, rs_stream_t stream) {
  RS_REQUIRE(reps && counts, "rs_embedding_gather_tables_rows_f32: null reps / counts");
  for (int j = 0; j < ntables; ++j)
    RS_REQUIRE(reps[j] && counts[j], "rs_embedding_gather_tables_rows_f32: null rep / count (table %d)", j);
  return gather_tables(ntables, tables, num_rows, ids, nullptr, n, outs, dim, bad_ids, stream, reps, counts);
}

int rs_embedding_gather_tables_ids_f32(int ntables, const float* const* tables, const int64_t* num_rows,
                                       const int64_t* const* dids, const int64_t* n, float* const* outs,
                                       int64_t dim, int32_t* bad_ids, rs_stream_t stream) {
  RS_REQUIRE(dim == 32 || dim == 64 || dim == 128, "rs_embedding_gather_tables_ids_f32: dim must be 32, 64 or 128");
  return gather_tables(ntables, tables, num_rows, dids, nullptr, n, outs, dim, bad_ids, stream, nullptr, nullptr,
                       true);
}

int rs_multi_embedding_gather_f32(const float* const* tables, const int64_t* num_rows, int nfeat,
                                  int64_t E, const int64_t* ids, int64_t B, const float* dense,
                                  int64_t nd, float* x0, int64_t ld, int32_t* bad_ids,
                                  rs_stream_t stream) {
  RS_REQUIRE(nfeat >= 0 && E > 0 && B >= 0 && nd >= 0, "rs_multi_embedding_gather_f32: bad sizes");
  RS_REQUIRE(E % 4 == 0 && ld % 4 == 0 && ld >= nfeat * E + nd, "rs_multi_embedding_gather_f32: layout");
  RS_REQUIRE(x0 && (nfeat == 0 || (tables && num_rows && ids)) && (nd == 0 || dense),
             "rs_multi_embedding_gather_f32: null");
  if (B == 0) return RS_OK;
  RS_REQUIRE(ld / 4 < (int64_t)1 << 30 && ceil_div(B, MG_RPB) < ((int64_t)1 << 31), "rs_multi_embedding_gather_f32: too large");
  hipLaunchKernelGGL(multi_gather_kernel, dim3((unsigned)ceil_div(ld / 4, 256), (unsigned)ceil_div(B, MG_RPB)),
                     dim3(256), 0, as_stream(stream), tables, num_rows, nfeat, E, ids, B, dense, nd, x0, ld, bad_ids);
  return check_launch("multi_embedding_gather");
}

size_t rs_sparse_adagrad_workspace_bytes(int64_t n, int64_t dim, int64_t num_rows) {
  (void)num_rows;
  return sparse_ws_bytes(1, &n, dim);
}

int rs_sparse_adagrad_f32(float* table, float* accum, int64_t num_rows, int64_t dim,
                          const int64_t* ids, const float* grad_rows, int64_t n,
                          const int64_t* iteration, float lr0, float decay_rate,
                          int64_t decay_steps, float clipnorm, float epsilon, void* workspace,
                          size_t workspace_bytes, rs_stream_t stream) {
  return rs_sparse_adagrad_ld_f32(table, accum, num_rows, dim, ids, grad_rows, dim, n, iteration, lr0,
                                  decay_rate, decay_steps, clipnorm, epsilon, workspace, workspace_bytes,
                                  stream);
}

int rs_sparse_dedupe_planned_f32(const int64_t* ids, const float* grad_rows, int64_t grad_ld, int64_t n,
                                 int64_t num_rows, int64_t dim, const int32_t* order, const int32_t* starts,
                                 const int64_t* dids, const int64_t* nslots, int64_t* out_ids, float* out_rows,
                                 int64_t* out_count, float* sumsq, void* workspace, size_t workspace_bytes,
                                 rs_stream_t stream) {
  RS_REQUIRE(num_rows > 0 && dim > 0 && n >= 0 && grad_ld >= dim, "rs_sparse_dedupe_planned_f32: bad sizes");
  RS_REQUIRE(n < (int64_t)1 << 31 && (dim == 32 || dim == 64 || dim == 128 || dim == 256),
             "rs_sparse_dedupe_planned_f32: n < 2^31, dim 32, 64, 128 or 256");
  RS_REQUIRE(out_ids && out_rows && out_count && (n == 0 || (ids && grad_rows && order && starts && dids && nslots)),
             "rs_sparse_dedupe_planned_f32: null");
  RS_REQUIRE(aligned16(out_rows) && aligned16(grad_rows) && grad_ld % 4 == 0,
             "rs_sparse_dedupe_planned_f32: 16-byte rows");
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    RS_HIP(hipMemsetAsync(out_count, 0, sizeof(int64_t), st));
    if (sumsq) RS_HIP(hipMemsetAsync(sumsq, 0, sizeof(float), st));
    return RS_OK;
  }
  const size_t need = rs_sparse_dedupe_workspace_bytes(n, dim, num_rows);
  if (!workspace || workspace_bytes < need || need == 0) {
    set_error("rs_sparse_dedupe_planned_f32: workspace too small (%zu < %zu)", workspace_bytes, need);
    return RS_ERR_WORKSPACE;
  }
  // the same carve-up and passes as rs_sparse_dedupe_f32, with the sort, flags and scan replaced by
  // the plan's order (the prep pass writes the sorted pairs) and its run heads
  Carve w(workspace, rs_sparse_adagrad_workspace_bytes(n, dim, num_rows));
  w.take<int64_t>(n);
  w.take<int32_t>(n);
  int64_t* keys_out = w.take<int64_t>(n);
  int32_t* vals_out = w.take<int32_t>(n);
  double* part = w.take<double>(sumsq_blocks(n * dim));
  float* ssq = w.take<float>(4);
  float* frag = w.take<float>((size_t)n * dim);
  SparseJobs jobs{};
  jobs.nt = 1;
  jobs.ids[0] = ids;
  jobs.rows[0] = grad_rows;
  jobs.ld[0] = grad_ld;
  jobs.n[0] = n;
  jobs.num_rows[0] = num_rows;
  jobs.off[1] = n;
  jobs.kbits = key_bits(num_rows);
  jobs.order[0] = order;
  hipLaunchKernelGGL(sparse_prep_kernel, dim3((unsigned)ceil_div(n, 256), 1), dim3(256), 0, st, jobs, keys_out,
                     vals_out, nullptr);
  int rc = check_launch("dedupe_planned_prep");
  if (rc) return rc;
  if (sumsq) {  // the norm of the RAW rows (Keras clips before deduplicating)
    rc = launch_sumsq_2d(grad_rows, n, dim, grad_ld, part, 1.0, ssq, st);
    if (rc) return rc;
    hipLaunchKernelGGL(sumsq_to_f32_kernel, dim3(1), dim3(1), 0, st, ssq, sumsq);
    rc = check_launch("dedupe_planned_sumsq");
    if (rc) return rc;
  }
  const int nv = (int)ceil_div(dim, 64);
  const int kWin = sparse_window(n);
  const unsigned gw = (unsigned)ceil_div(ceil_div(n, kWin), 4);
  if (nv <= 1) hipLaunchKernelGGL((sparse_fragment_kernel<1>), dim3(gw), dim3(256), 0, st, keys_out, vals_out, jobs, n, dim, 0.f, kWin, frag);
  else if (nv <= 2) hipLaunchKernelGGL((sparse_fragment_kernel<2>), dim3(gw), dim3(256), 0, st, keys_out, vals_out, jobs, n, dim, 0.f, kWin, frag);
  else hipLaunchKernelGGL((sparse_fragment_kernel<4>), dim3(gw), dim3(256), 0, st, keys_out, vals_out, jobs, n, dim, 0.f, kWin, frag);
  rc = check_launch("dedupe_planned_fragment");
  if (rc) return rc;
  const int lph = (int)(dim / 4);
  const unsigned gh = (unsigned)ceil_div(ceil_div(n, 64 / lph), 4);
  if (lph == 8) hipLaunchKernelGGL((dedupe_heads_kernel<8>), dim3(gh), dim3(256), 0, st, starts, dids, nslots, n, dim, num_rows, kWin, frag, out_ids, out_rows, out_count);
  else if (lph == 16) hipLaunchKernelGGL((dedupe_heads_kernel<16>), dim3(gh), dim3(256), 0, st, starts, dids, nslots, n, dim, num_rows, kWin, frag, out_ids, out_rows, out_count);
  else if (lph == 32) hipLaunchKernelGGL((dedupe_heads_kernel<32>), dim3(gh), dim3(256), 0, st, starts, dids, nslots, n, dim, num_rows, kWin, frag, out_ids, out_rows, out_count);
  else hipLaunchKernelGGL((dedupe_heads_kernel<64>), dim3(gh), dim3(256), 0, st, starts, dids, nslots, n, dim, num_rows, kWin, frag, out_ids, out_rows, out_count);
  return check_launch("dedupe_heads");
}

// The stable ascending order of R sorted runs of distinct ids concatenated (the deduplicating
// exchange's gathered ids: every rank's unique ids ascending, rank order): element j of run r goes to
// position j + sum over earlier runs of their ids <= its id + sum over later runs of their ids < its id
// (binary searches), so equal ids keep rank order — the stable sort's permutation, without a sort.
constexpr int MR_MAXR = 64;
struct MergeRuns {
  int64_t off[MR_MAXR + 1];
  int nr;
};
__device__ __forceinline__ int64_t mr_count(const int64_t* __restrict__ a, int64_t lo, int64_t hi, int64_t v,
                                            bool le) {  // elements of a[lo, hi) < v (<= v when le)
  int64_t l = lo, h = hi;
  while (l < h) {
    const int64_t m = (l + h) >> 1;
    const bool go = le ? a[m] <= v : a[m] < v;
    if (go) l = m + 1;
    else h = m;
  }
  return l - lo;
}
// 8 lanes per element: lane g of the group searches runs g, g + 8, ... (the searches of one element
// run side by side instead of one after another), then the group sums its counts
__global__ __launch_bounds__(256) void merge_runs_order_kernel(const int64_t* __restrict__ ids, MergeRuns mr,
                                                               int32_t* __restrict__ order) {
  const int g = threadIdx.x & 7;
  const int64_t n = mr.off[mr.nr];
  const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 3;
  const int64_t p = p0 < n ? p0 : n - 1;  // (every lane takes part in the group's shuffles)
  int r = 0;
  while (r + 1 < mr.nr && p >= mr.off[r + 1]) ++r;
  const int64_t v = ids[p];
  int64_t pos = 0;
  for (int q = g; q < mr.nr; q += 8)
    if (q != r) pos += mr_count(ids, mr.off[q], mr.off[q + 1], v, q < r);
  pos += __shfl_xor(pos, 1, 64);
  pos += __shfl_xor(pos, 2, 64);
  pos += __shfl_xor(pos, 4, 64);
  if (g == 0 && p0 < n) order[pos + p - mr.off[r]] = (int32_t)p;
}

int rs_merge_runs_order_i64(const int64_t* ids, const int64_t* run_off, int nruns, int32_t* order,
                            rs_stream_t stream) {
  RS_REQUIRE(nruns >= 1 && nruns <= MR_MAXR && run_off, "rs_merge_runs_order_i64: 1..%d runs", MR_MAXR);
  MergeRuns mr{};
  mr.nr = nruns;
  for (int r = 0; r <= nruns; ++r) {
    mr.off[r] = run_off[r];
    RS_REQUIRE(r == 0 ? run_off[0] == 0 : run_off[r] >= run_off[r - 1], "rs_merge_runs_order_i64: bad run offsets");
  }
  const int64_t n = mr.off[nruns];
  RS_REQUIRE(n < (int64_t)1 << 31, "rs_merge_runs_order_i64: n < 2^31");
  if (n == 0) return RS_OK;
  RS_REQUIRE(ids && order, "rs_merge_runs_order_i64: null");
  hipLaunchKernelGGL(merge_runs_order_kernel, dim3((unsigned)ceil_div(n * 8, 256)), dim3(256), 0, as_stream(stream),
                     ids, mr, order);
  return check_launch("merge_runs_order");
}

static int sparse_update(float* table, float* accum, int64_t num_rows, int64_t dim, const int64_t* ids,
                         const float* grad_rows, int64_t grad_ld, int64_t n, const int64_t* iteration, float lr0,
                         float decay_rate, int64_t decay_steps, float clipnorm, float epsilon,
                         const float* sumsq_ext, void* workspace, size_t workspace_bytes, rs_stream_t stream);

int rs_sparse_adagrad_ld_f32(float* table, float* accum, int64_t num_rows, int64_t dim,
                             const int64_t* ids, const float* grad_rows, int64_t grad_ld, int64_t n,
                             const int64_t* iteration, float lr0, float decay_rate,
                             int64_t decay_steps, float clipnorm, float epsilon, void* workspace,
                             size_t workspace_bytes, rs_stream_t stream) {
  return sparse_update(table, accum, num_rows, dim, ids, grad_rows, grad_ld, n, iteration, lr0, decay_rate,
                       decay_steps, clipnorm, epsilon, nullptr, workspace, workspace_bytes, stream);
}

int rs_sparse_adagrad_sumsq_f32(float* table, float* accum, int64_t num_rows, int64_t dim,
                                const int64_t* ids, const float* grad_rows, int64_t grad_ld, int64_t n,
                                const float* sumsq, const int64_t* iteration, float lr0, float decay_rate,
                                int64_t decay_steps, float clipnorm, float epsilon, void* workspace,
                                size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(sumsq || clipnorm <= 0.f, "rs_sparse_adagrad_sumsq_f32: sumsq is required when clipping");
  return sparse_update(table, accum, num_rows, dim, ids, grad_rows, grad_ld, n, iteration, lr0, decay_rate,
                       decay_steps, clipnorm, epsilon, sumsq, workspace, workspace_bytes, stream);
}

size_t rs_sparse_dedupe_workspace_bytes(int64_t n, int64_t dim, int64_t num_rows) {
  size_t sb = 0;
  if (rocprim::exclusive_scan(nullptr, sb, (const int32_t*)nullptr, (int32_t*)nullptr, 0, (size_t)(n > 0 ? n : 1),
                              rocprim::plus<int32_t>(), (hipStream_t)0) != hipSuccess)
    return 0;
  Carve c(nullptr, 0);
  c.take<char>(rs_sparse_adagrad_workspace_bytes(n, dim, num_rows));
  c.take<int32_t>((size_t)(n > 0 ? n : 1));
  c.take<int32_t>((size_t)(n > 0 ? n : 1));
  c.take<char>(sb);
  return c.off + 256;
}

int rs_sparse_dedupe_f32(const int64_t* ids, const float* grad_rows, int64_t grad_ld, int64_t n, int64_t num_rows,
                         int64_t dim, int64_t* out_ids, float* out_rows, int64_t* out_count, float* sumsq,
                         void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(num_rows > 0 && dim > 0 && n >= 0 && grad_ld >= dim, "rs_sparse_dedupe_f32: bad sizes");
  RS_REQUIRE(n < (int64_t)1 << 31 && dim <= 256, "rs_sparse_dedupe_f32: n < 2^31, dim <= 256");
  RS_REQUIRE(out_ids && out_rows && out_count && (n == 0 || (ids && grad_rows)), "rs_sparse_dedupe_f32: null");
  RS_REQUIRE(dim <= 64 || (dim % (dim <= 128 ? 2 : 4) == 0 && aligned16(out_rows)),
             "rs_sparse_dedupe_f32: dim > 64 must be a multiple of 2 (4 above 128), out_rows 16-byte aligned");
  hipStream_t st = as_stream(stream);
  if (n == 0) {
    RS_HIP(hipMemsetAsync(out_count, 0, sizeof(int64_t), st));
    if (sumsq) RS_HIP(hipMemsetAsync(sumsq, 0, sizeof(float), st));
    return RS_OK;
  }
  const size_t need = rs_sparse_dedupe_workspace_bytes(n, dim, num_rows);
  if (!workspace || workspace_bytes < need || need == 0) {
    set_error("rs_sparse_dedupe_f32: workspace too small (%zu < %zu)", workspace_bytes, need);
    return RS_ERR_WORKSPACE;
  }
  size_t tb = 0;
  if (sort_temp_bytes(n, &tb) != RS_OK) {
    set_error("rs_sparse_dedupe_f32: rocprim temp query failed");
    return RS_ERR_HIP;
  }
  Carve c(workspace, workspace_bytes);
  char* sparse_ws = c.take<char>(rs_sparse_adagrad_workspace_bytes(n, dim, num_rows));
  int32_t* flags = c.take<int32_t>((size_t)n);
  int32_t* slots = c.take<int32_t>((size_t)n);
  size_t sb = 0;
  if (rocprim::exclusive_scan(nullptr, sb, flags, slots, 0, (size_t)n, rocprim::plus<int32_t>(), st) != hipSuccess) {
    set_error("rs_sparse_dedupe_f32: rocprim scan temp query failed");
    return RS_ERR_HIP;
  }
  char* scan_temp = c.take<char>(sb);
  Carve w(sparse_ws, rs_sparse_adagrad_workspace_bytes(n, dim, num_rows));  // the update's own carve-up
  int64_t* keys_in = w.take<int64_t>(n);
  int32_t* vals_in = w.take<int32_t>(n);
  int64_t* keys_out = w.take<int64_t>(n);
  int32_t* vals_out = w.take<int32_t>(n);
  double* part = w.take<double>(sumsq_blocks(n * dim));
  float* ssq = w.take<float>(4);
  float* frag = w.take<float>((size_t)n * dim);
  char* temp = w.take<char>(tb);
  SparseJobs jobs{};  // one table, no padding: keys = ids (num_rows for invalid ones)
  jobs.nt = 1;
  jobs.ids[0] = ids;
  jobs.rows[0] = grad_rows;
  jobs.ld[0] = grad_ld;
  jobs.n[0] = n;
  jobs.num_rows[0] = num_rows;
  jobs.off[1] = n;
  jobs.kbits = key_bits(num_rows);
  hipLaunchKernelGGL(sparse_prep_kernel, dim3((unsigned)ceil_div(n, 256), 1), dim3(256), 0, st, jobs, keys_in, vals_in,
                     nullptr);
  int rc = check_launch("dedupe_prep");
  if (rc) return rc;
  hipError_t e = sort_pairs_i64(temp, tb, keys_in, keys_out, vals_in, vals_out, n, key_bits(num_rows), st);
  if (e != hipSuccess) {
    set_error("rs_sparse_dedupe_f32: radix sort failed: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  if (sumsq) {  // the norm of the RAW rows (Keras clips before deduplicating)
    rc = launch_sumsq_2d(grad_rows, n, dim, grad_ld, part, 1.0, ssq, st);
    if (rc) return rc;
    hipLaunchKernelGGL(sumsq_to_f32_kernel, dim3(1), dim3(1), 0, st, ssq, sumsq);
    rc = check_launch("dedupe_sumsq");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(dedupe_flags_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, st, keys_out, n, num_rows,
                     flags);
  rc = check_launch("dedupe_flags");
  if (rc) return rc;
  e = rocprim::exclusive_scan(scan_temp, sb, flags, slots, 0, (size_t)n, rocprim::plus<int32_t>(), st);
  if (e != hipSuccess) {
    set_error("rs_sparse_dedupe_f32: scan failed: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  const int nv = (int)ceil_div(dim, 64);
  const int kWin = sparse_window(n);
  const unsigned gw = (unsigned)ceil_div(ceil_div(n, kWin), 4);
  const unsigned ga = (unsigned)ceil_div(n, 4);
#define RS_DEDUPE(NV)                                                                                        \
  hipLaunchKernelGGL((sparse_fragment_kernel<NV>), dim3(gw), dim3(256), 0, st, keys_out, vals_out, jobs, n, dim, \
                     0.f, kWin, frag);                                                                         \
  rc = check_launch("dedupe_fragment");                                                                      \
  if (rc) return rc;                                                                                         \
  hipLaunchKernelGGL((dedupe_apply_kernel<NV>), dim3(ga), dim3(256), 0, st, keys_out, frag, n, dim, num_rows, kWin, \
                     slots, out_ids, out_rows, out_count);
  if (nv <= 1) { RS_DEDUPE(1) }
  else if (nv <= 2) { RS_DEDUPE(2) }
  else { RS_DEDUPE(4) }
#undef RS_DEDUPE
  return check_launch("dedupe_apply");
}

static int sparse_update(float* table, float* accum, int64_t num_rows, int64_t dim, const int64_t* ids,
                         const float* grad_rows, int64_t grad_ld, int64_t n, const int64_t* iteration, float lr0,
                         float decay_rate, int64_t decay_steps, float clipnorm, float epsilon,
                         const float* sumsq_ext, void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(num_rows > 0 && dim > 0 && n >= 0, "rs_sparse_adagrad_f32: bad sizes");
  RS_REQUIRE(grad_ld >= dim, "rs_sparse_adagrad_f32: grad_ld must be >= dim");
  RS_REQUIRE(n < (int64_t)1 << 31, "rs_sparse_adagrad_f32: n too large");
  RS_REQUIRE(table && accum && iteration && (n == 0 || (ids && grad_rows)),
             "rs_sparse_adagrad_f32: null pointer");
  RS_REQUIRE(decay_steps > 0, "rs_sparse_adagrad_f32: decay_steps must be > 0");
  RS_REQUIRE(dim <= 256, "rs_sparse_adagrad_f32: dim must be <= 256");
  // the row update moves 2 / 4 contiguous floats per lane above 64 / 128 columns
  RS_REQUIRE(dim <= 64 || (dim % (dim <= 128 ? 2 : 4) == 0 && aligned16(table) && aligned16(accum)),
             "rs_sparse_adagrad_f32: dim > 64 must be a multiple of 2 (4 above 128), tables 16-byte aligned");
  if (n == 0) return RS_OK;
  SparseJobs jobs{};
  jobs.nt = 1;
  jobs.ids[0] = ids;
  jobs.rows[0] = grad_rows;
  jobs.ld[0] = grad_ld;
  jobs.n[0] = n;
  jobs.num_rows[0] = num_rows;
  jobs.table[0] = table;
  jobs.accum[0] = accum;
  jobs.sumsq[0] = sumsq_ext;
  return sparse_run(jobs, dim, iteration, lr0, decay_rate, decay_steps, clipnorm, epsilon,
                    clipnorm > 0.f && sumsq_ext, workspace, workspace_bytes, as_stream(stream));
}

size_t rs_sparse_adagrad_multi_workspace_bytes(int ntables, const int64_t* n, int64_t dim) {
  if (ntables < 1 || ntables > SP_MAXT || !n) return 0;
  return sparse_ws_bytes(ntables, n, dim);
}

static int sparse_multi_impl(int ntables, float* const* tables, float* const* accums, const int64_t* num_rows,
                             int64_t dim, const int64_t* const* ids, const float* const* grad_rows,
                             const int64_t* grad_ld, const int64_t* n, const float* const* sumsq,
                             const int64_t* iteration, float lr0, float decay_rate, int64_t decay_steps,
                             float clipnorm, float epsilon, void* workspace, size_t workspace_bytes,
                             rs_stream_t stream, int64_t* iter_inc, const int32_t* const* orders = nullptr,
                             const int32_t* const* starts = nullptr, const int64_t* const* dids = nullptr,
                             const int64_t* const* nslots = nullptr) {
  RS_REQUIRE(ntables >= 1 && ntables <= SP_MAXT, "rs_sparse_adagrad_multi_f32: 1..%d tables", SP_MAXT);
  RS_REQUIRE(tables && accums && num_rows && ids && grad_rows && grad_ld && n && iteration,
             "rs_sparse_adagrad_multi_f32: null array");
  RS_REQUIRE(dim > 0 && dim <= 256, "rs_sparse_adagrad_multi_f32: dim must be in 1..256");
  RS_REQUIRE(decay_steps > 0, "rs_sparse_adagrad_multi_f32: decay_steps must be > 0");
  SparseJobs jobs{};
  jobs.nt = ntables;
  int64_t total = 0;
  for (int k = 0; k < ntables; ++k) {
    RS_REQUIRE(num_rows[k] > 0 && n[k] >= 0 && n[k] < (int64_t)1 << 31 && grad_ld[k] >= dim,
               "rs_sparse_adagrad_multi_f32: bad sizes (table %d)", k);
    RS_REQUIRE(tables[k] && accums[k] && (n[k] == 0 || (ids[k] && grad_rows[k])),
               "rs_sparse_adagrad_multi_f32: null pointer (table %d)", k);
    RS_REQUIRE(dim <= 64 || (dim % (dim <= 128 ? 2 : 4) == 0 && aligned16(tables[k]) && aligned16(accums[k])),
               "rs_sparse_adagrad_multi_f32: dim > 64 must be a multiple of 2 (4 above 128), tables 16-byte "
               "aligned (table %d)", k);
    RS_REQUIRE(clipnorm <= 0.f || !sumsq || sumsq[k], "rs_sparse_adagrad_multi_f32: sumsq[%d] is null", k);
    RS_REQUIRE(!orders || orders[k] || n[k] == 0, "rs_sparse_adagrad_multi: orders[%d] is null", k);
    if (starts) {
      RS_REQUIRE(orders && starts[k] && dids[k] && nslots[k], "rs_sparse_adagrad_multi: null plan heads (table %d)", k);
      RS_REQUIRE(aligned16(tables[k]) && aligned16(accums[k]), "rs_sparse_adagrad_multi: 16-byte tables (table %d)", k);
      jobs.hstart[k] = starts[k];
      jobs.hdid[k] = dids[k];
      jobs.hcount[k] = nslots[k];
    }
    jobs.ids[k] = ids[k];
    jobs.order[k] = orders ? orders[k] : nullptr;
    jobs.rows[k] = grad_rows[k];
    jobs.ld[k] = grad_ld[k];
    jobs.n[k] = n[k];
    jobs.num_rows[k] = num_rows[k];
    jobs.table[k] = tables[k];
    jobs.accum[k] = accums[k];
    jobs.sumsq[k] = sumsq ? sumsq[k] : nullptr;
    total += n[k];
  }
  RS_REQUIRE(total + (int64_t)ntables * 64 < (int64_t)1 << 31, "rs_sparse_adagrad_multi_f32: too many rows");
  if (total == 0) return iter_inc ? rs_iteration_increment(iter_inc, stream) : RS_OK;
  return sparse_run(jobs, dim, iteration, lr0, decay_rate, decay_steps, clipnorm, epsilon,
                    clipnorm > 0.f && sumsq != nullptr, workspace, workspace_bytes, as_stream(stream), iter_inc);
}

int rs_sparse_adagrad_multi_f32(int ntables, float* const* tables, float* const* accums, const int64_t* num_rows,
                                int64_t dim, const int64_t* const* ids, const float* const* grad_rows,
                                const int64_t* grad_ld, const int64_t* n, const float* const* sumsq,
                                const int64_t* iteration, float lr0, float decay_rate, int64_t decay_steps,
                                float clipnorm, float epsilon, void* workspace, size_t workspace_bytes,
                                rs_stream_t stream) {
  return sparse_multi_impl(ntables, tables, accums, num_rows, dim, ids, grad_rows, grad_ld, n, sumsq, iteration, lr0,
                           decay_rate, decay_steps, clipnorm, epsilon, workspace, workspace_bytes, stream, nullptr);
}

int rs_sparse_adagrad_multi_step_f32(int ntables, float* const* tables, float* const* accums, const int64_t* num_rows,
                                     int64_t dim, const int64_t* const* ids, const float* const* grad_rows,
                                     const int64_t* grad_ld, const int64_t* n, const float* const* sumsq,
                                     int64_t* iteration, float lr0, float decay_rate, int64_t decay_steps,
                                     float clipnorm, float epsilon, void* workspace, size_t workspace_bytes,
                                     rs_stream_t stream) {
  RS_REQUIRE(iteration, "rs_sparse_adagrad_multi_step_f32: null iteration");
  return sparse_multi_impl(ntables, tables, accums, num_rows, dim, ids, grad_rows, grad_ld, n, sumsq, iteration, lr0,
                           decay_rate, decay_steps, clipnorm, epsilon, workspace, workspace_bytes, stream, iteration);
}

int rs_sparse_adagrad_multi_step_ordered_f32(int ntables, float* const* tables, float* const* accums,
                                             const int64_t* num_rows, int64_t dim, const int64_t* const* ids,
                                             const float* const* grad_rows, const int64_t* grad_ld, const int64_t* n,
                                             const float* const* sumsq, int64_t* iteration, float lr0,
                                             float decay_rate, int64_t decay_steps, float clipnorm, float epsilon,
                                             const int32_t* const* orders, void* workspace, size_t workspace_bytes,
                                             rs_stream_t stream) {
  RS_REQUIRE(iteration && orders, "rs_sparse_adagrad_multi_step_ordered_f32: null iteration / orders");
  return sparse_multi_impl(ntables, tables, accums, num_rows, dim, ids, grad_rows, grad_ld, n, sumsq, iteration, lr0,
                           decay_rate, decay_steps, clipnorm, epsilon, workspace, workspace_bytes, stream, iteration,
                           orders);
}

int rs_sparse_adagrad_multi_step_planned_f32(int ntables, float* const* tables, float* const* accums,
                                             const int64_t* num_rows, int64_t dim, const int64_t* const* ids,
                                             const float* const* grad_rows, const int64_t* grad_ld, const int64_t* n,
                                             const float* const* sumsq, int64_t* iteration, float lr0,
                                             float decay_rate, int64_t decay_steps, float clipnorm, float epsilon,
                                             const int32_t* const* orders, const int32_t* const* starts,
                                             const int64_t* const* dids, const int64_t* const* nslots,
                                             void* workspace, size_t workspace_bytes, rs_stream_t stream) {
  RS_REQUIRE(iteration && orders && starts && dids && nslots,
             "rs_sparse_adagrad_multi_step_planned_f32: null iteration / orders / plan heads");
  return sparse_multi_impl(ntables, tables, accums, num_rows, dim, ids, grad_rows, grad_ld, n, sumsq, iteration, lr0,
                           decay_rate, decay_steps, clipnorm, epsilon, workspace, workspace_bytes, stream, iteration,
                           orders, starts, dids, nslots);
}

}  // extern "C"
