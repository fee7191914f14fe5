// nc_det.hip -- NC_DETERMINISTIC grid-gradient scatter (SURVEY.md §8b "Determinism").
//
// The default backward scatters the trilinear grid gradient with float atomics inside
// k_mlp_dx (nc_grid.h), whose summation order varies run to run.  With
// NC_DETERMINISTIC, k_mlp_dx stores each point's feature gradient instead
// (MlpCtx::dfeat) and this file reduces them in a fixed order:
//   k_det_keys    entry (job, point, corner) -> key (job << vbits | voxel), weight, and
//                 the first sort pass's digit counts (one workgroup = one radix tile)
//   radix sort    a stable LSD radix sort of (key, entry id), 8-11 bits per pass, written
//                 here (k_rs_hist -> k_rs_scan -> k_rs_scatter): the entries of one voxel
//                 end up adjacent, in ascending (point, corner) order
//   k_det_runs /  each voxel run is summed (w * d feature, channel per lane) in
//   k_det_join    entry order, 16 entries per half-wave, boundary pieces joined in
//                 order; one writer per voxel (no atomics)
// The order is the reference's own: ATen's CPU grid_sampler_3d_backward walks points
// in order and adds each point's 8 corner contributions (gInp += gOut * w), and a
// voxel is a corner of a point at most once.
#include "nc_device.h"
#include "nc_internal.h"

namespace nc {

__device__ __forceinline__ Job job_of(const MlpCtx& m, int j) {
  return j == 0 ? m.jobs[0] : (j == 1 ? m.jobs[1] : m.jobs[2]);
}
__device__ __forceinline__ nc_grid grid_of(const MlpCtx& m, int kind) {
  return kind == 0 ? m.grids[0] : kind == 1 ? m.grids[1] : kind == 2 ? m.grids[2] : m.grids[3];
}

// K: uint32_t keys when job and voxel bits fit (vbits + 2 <= 32: every BASELINE grid,
// C5's 204M-voxel grids included), else uint64_t; the key buffers are sized for 64 bits
// a point's 8 entries are contiguous: 16-byte stores (the first sort pass takes the entry
// id from the position, so no id array is written here)
template <typename T>
__device__ __forceinline__ void store8(T* dst, const T (&v)[8]) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "4- or 8-byte entries");
  if constexpr (sizeof(T) == 4) {
    uint4* o = reinterpret_cast<uint4*>(dst);
    o[0] = make_uint4(__builtin_bit_cast(uint32_t, v[0]), __builtin_bit_cast(uint32_t, v[1]),
                      __builtin_bit_cast(uint32_t, v[2]), __builtin_bit_cast(uint32_t, v[3]));
    o[1] = make_uint4(__builtin_bit_cast(uint32_t, v[4]), __builtin_bit_cast(uint32_t, v[5]),
                      __builtin_bit_cast(uint32_t, v[6]), __builtin_bit_cast(uint32_t, v[7]));
  } else {
    ulonglong2* o = reinterpret_cast<ulonglong2*>(dst);
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = make_ulonglong2(v[2 * q], v[2 * q + 1]);
  }
}

// radix sort tiles (the sort itself is below, after the run kernels)
constexpr int RS_THREADS = 256;
#ifndef NC_RS_ROUNDS
#define NC_RS_ROUNDS 8  // 2,048-key tiles: 564 workgroups at C2 (16: 282, 5 us slower; 4, 32 slower still)
#endif
constexpr int RS_ROUNDS = NC_RS_ROUNDS;
constexpr int RS_TILE = RS_THREADS * RS_ROUNDS;
constexpr int RS_MAX_BITS = 11;

// The first sort pass's digit counts are formed here: a workgroup's 256 points x 8
// corners are exactly one radix tile (RS_TILE) because each job's points are padded to
// a multiple of 256 (DetBufs::ppad; the padding entries carry the invalid key), so the
// tile's row hist[tile][digit] is written here and the pass needs no k_rs_hist.
constexpr int DET_TILE_POINTS = 256;
constexpr bool KEYS_HIST = RS_TILE == 8 * DET_TILE_POINTS;
template <typename K>
__global__ void __launch_bounds__(DET_TILE_POINTS) k_det_keys(const MlpCtx m, DetBufs d) {
  __shared__ uint32_t cnt[1 << RS_MAX_BITS];
  K* keys = reinterpret_cast<K*>(d.key[0]);
  const int j = blockIdx.y;
  const int64_t p = (int64_t)blockIdx.x * DET_TILE_POINTS + threadIdx.x;  // < ppad
  const int bins = 1 << d.sort_bits;
  for (int b = threadIdx.x; b < bins; b += DET_TILE_POINTS) cnt[b] = 0u;
  const Job job = job_of(m, j);
  const K invalid = (K)((uint64_t(1) << (d.vbits + 2)) - 1);
  const int64_t e0 = ((int64_t)j * d.ppad + p) * 8;
  K kk[8];
  float ww[8];
  if (!job.need_grid || p >= m.P) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      kk[k] = invalid;
      ww[k] = 0.f;
    }
  } else {
    const nc_grid G = grid_of(m, job.kind);
    const float4 n = m.xyz[(int64_t)job.slot * m.P + p];
    const float xyz[3] = {n.x, n.y, n.z};
    Corners c;
    make_corners(G, xyz, c);
    const uint64_t H = (uint64_t)G.dims[1], W = (uint64_t)G.dims[2];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t x = (uint64_t)(c.x0 + (k & 1)), y = (uint64_t)(c.y0 + ((k >> 1) & 1)),
                     z = (uint64_t)(c.z0 + (k >> 2));
      const bool in = (c.inb >> k) & 1u;
      kk[k] = in ? (K)(((uint64_t)j << d.vbits) | ((z * H + y) * W + x)) : invalid;
      ww[k] = c.w[k];
    }
  }
  store8(keys + e0, kk);
  store8(d.w + e0, ww);
  if constexpr (!KEYS_HIST) return;  // (other tile sizes: k_rs_hist counts)
  __syncthreads();  // counts zeroed
#pragma unroll
  for (int k = 0; k < 8; ++k) atomicAdd(&cnt[(int)((uint64_t)kk[k] & (uint64_t)(bins - 1))], 1u);
  __syncthreads();
  uint32_t* hist = reinterpret_cast<uint32_t*>(d.temp) +
                   ((int64_t)j * (d.ppad / DET_TILE_POINTS) + blockIdx.x) * bins;
  for (int b = threadIdx.x; b < bins; b += DET_TILE_POINTS) hist[b] = cnt[b];
}

// The sorted entries are cut into sub-chunks of DSUB = 16, one per half-wave (lane =
// channel), eight per workgroup (a chunk of DCH = 8 DSUB entries).  A voxel's run of
// entries is summed in entry order, one sub-chunk at a time: k_det_runs sums every run
// piece of its sub-chunk in registers and parks the sums in LDS; a run that crosses
// sub-chunk boundaries inside the chunk is then added up, piece by piece in sub-chunk
// order, by the half-wave where it starts, and every run that ends inside the chunk is
// written straight to the gradient.  A run that crosses a chunk boundary leaves its
// chunk's piece in DetBufs::part (slot 0: the chunk's first run, slot 1: its last), and
// k_det_join, in the chunk where the run starts, adds the pieces up in chunk order.
// Every run has one writer, a hot voxel's thousands of entries are summed 16 at a time
// in parallel, and the order is fixed by the sort: bit-identical from run to run.
// (16-entry sub-chunks: 70 VGPRs and 17 KB of LDS, 7 waves per SIMD where 32 entries
// held 4; the in-chunk join keeps the extra boundaries out of k_det_join.)
constexpr int DSUB = DET_DSUB;
constexpr int DCH = 8 * DSUB;
static_assert(DSUB == 16 || DSUB == 32, "a sub-chunk fits one half-wave");

__device__ __forceinline__ uint32_t shfl_key(uint32_t v, int src) { return __shfl(v, src, 32); }
__device__ __forceinline__ uint64_t shfl_key(uint64_t v, int src) {
  const unsigned lo = __shfl((unsigned)(v & 0xffffffffu), src, 32);
  const unsigned hi = __shfl((unsigned)(v >> 32), src, 32);
  return ((uint64_t)hi << 32) | lo;
}

// the summed run of voxel key k0 added to its gradient row.  Read-add-write without an
// atomic: every voxel of a grid is the key of at most one run (each grid belongs to one
// job: a decoder samples its own grid with grad, Plan), so the run has one writer.  The
// add (not a store) keeps the accumulate contract of nicecore.h: sparse rows collect
// several forward/backward calls until nc_sparse_rows_clear, and a caller's dense
// gradient buffer keeps what was in it, exactly as the float-atomic path does
__device__ __forceinline__ float* det_dst(const MlpCtx& m, const DetBufs& d, uint64_t k0, int ch) {
  const int j = (int)(k0 >> d.vbits);
  const uint64_t v = k0 & ((uint64_t(1) << d.vbits) - 1);
  const nc_grid G = grid_of(m, job_of(m, j).kind);
  if (G.grad_rows) {  // sparse gradient rows (claimed by the forward)
    const int r = G.grad_rows[v];
    return r >= 0 ? G.grad + (int64_t)r * 32 + ch : nullptr;
  }
  const int64_t H = G.dims[1], W = G.dims[2];
  if (G.grad_stride[0] == 1 && G.grad_stride[3] == 32 && G.grad_stride[2] == 32 * W && G.grad_stride[1] == 32 * W * H)
    return G.grad + 32 * (int64_t)v + ch;  // packed channels-last gradient: row v
  const int64_t x = (int64_t)(v % W), y = (int64_t)((v / W) % H), z = (int64_t)(v / (W * H));
  return G.grad + z * G.grad_stride[1] + y * G.grad_stride[2] + x * G.grad_stride[3] + (int64_t)ch * G.grad_stride[0];
}

// The gradient row of voxel key k0 resolved through per-job descriptors read once per
// launch (job and grid are uniform there, so they sit in scalar registers): the run loop
// then selects among them per run instead of indexing the kernel argument with a
// per-lane job, which the compiler turns into dependent vector loads of the argument.
struct DetRows {
  float* grad[3];
  const int32_t* rows[3];  // sparse gradient rows, or nullptr: dense channels-last rows
  bool fast;               // every job with a grid gradient has sparse or packed dense rows
  bool any_rows;           // some job has sparse rows (else no row-id loads at all)
};
__device__ __forceinline__ DetRows det_rows(const MlpCtx& m) {
  DetRows r;
  r.fast = true;
  r.any_rows = false;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const Job job = job_of(m, j);
    const nc_grid G = grid_of(m, job.kind);
    const int64_t H = G.dims[1], W = G.dims[2];
    r.grad[j] = G.grad;
    r.rows[j] = G.grad_rows;
    const bool packed = G.grad_stride[0] == 1 && G.grad_stride[3] == 32 && G.grad_stride[2] == 32 * W &&
                        G.grad_stride[1] == 32 * W * H;
    r.fast = r.fast && (!job.need_grid || G.grad_rows || packed);
    r.any_rows = r.any_rows || (job.need_grid && G.grad_rows);
  }
  return r;
}

// half-wave = sub-chunk s (entries [32 s, 32 s + 32)), lane = channel.  The run sums are
// formed in registers, parked in LDS, then written by one loop over the runs.  Every load
// is unconditional (clamped index, result selected afterwards): a load under a branch is
// issued alone and waited for, which made each of the 32 row gathers a serial latency.
template <typename K>
__global__ void __launch_bounds__(256) k_det_runs(const MlpCtx m, DetBufs d, int64_t n) {
  __shared__ float racc[8][DSUB][32];
  __shared__ K rkey[8][DSUB];
  __shared__ K rnext[8];  // the key after each sub-chunk (invalid past the end)
  __shared__ int rcnt[8];  // runs of each sub-chunk
  const int hw = threadIdx.x >> 5, ch = threadIdx.x & 31;
  const int64_t s = (int64_t)blockIdx.x * 8 + hw;
  const int64_t e0 = s * DSUB;
  const int cnt = e0 >= n ? 0 : (int)(n - e0 < DSUB ? n - e0 : DSUB);
  const K* key = reinterpret_cast<const K*>(d.sorted ? d.key[1] : d.key[0]);  // select: a runtime index into the argument copies it to scratch
  const uint32_t* val = d.sorted ? d.val[1] : d.val[0];
  const K invalid = (K)((uint64_t(1) << (d.vbits + 2)) - 1);
  // the sub-chunk's entries, one per lane (coalesced), and the neighbours' keys
  const int64_t ec = e0 + ch < n ? e0 + ch : n - 1;
  const K kraw = key[ec];
  const uint32_t eraw = val[ec];
  const K kprev = key[e0 > 0 && e0 <= n ? e0 - 1 : 0];
  const K knext = key[e0 + cnt < n ? e0 + cnt : 0];
  const K myk = ch < cnt ? kraw : invalid;
  const uint32_t ent = myk != invalid ? eraw : 0u;  // an invalid corner (outside the grid, or a
  const float wraw = d.w[ent];                      // job without a grid gradient: sorted to
  const float myw = myk != invalid ? wraw : 0.f;    // the end) reads row 0 times weight 0 into
                                                    // a run that is never written
  // every entry's feature-gradient row in flight at once, then weighted.  Entry id / 8 =
  // job * ppad + point, the d features are [job][P][32] (no padding): this lane's row
  const uint32_t q = ent >> 3, jq = (uint32_t)(q >= d.ppad) + (uint32_t)(q >= 2 * d.ppad);
  const int32_t frow = (int32_t)(q - jq * (uint32_t)(d.ppad - m.P));
  float v[DSUB];
#pragma unroll
  for (int i = 0; i < DSUB; ++i) v[i] = m.dfeat[(int64_t)__shfl(frow, i, 32) * 32 + ch];
#pragma unroll
  for (int i = 0; i < DSUB; ++i) v[i] = v[i] * __shfl(myw, i, 32);
  int nr = 0;
  if (cnt > 0) {
    K cur = shfl_key(myk, 0);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < DSUB; ++i) {
      if (i < cnt) {
        const K k = shfl_key(myk, i);
        if (k != cur) {
          racc[hw][nr][ch] = acc;
          if (ch == 0) rkey[hw][nr] = cur;
          ++nr;
          cur = k;
          acc = 0.f;
        }
        acc = acc + v[i];
      }
    }
    racc[hw][nr][ch] = acc;
    if (ch == 0) rkey[hw][nr] = cur;
    ++nr;
  }
  const K prevk = e0 > 0 ? kprev : invalid;
  const K nextk = e0 + cnt < n ? knext : invalid;
  if (ch == 0) {
    rcnt[hw] = nr;
    rnext[hw] = cnt > 0 ? nextk : invalid;
  }
  __syncthreads();
  if (cnt == 0) return;
  // runs crossing this sub-chunk's ends: the first continues an earlier run (cin), the last
  // goes on into the next sub-chunk (cout)
  const K kf = rkey[hw][0], kl = rkey[hw][nr - 1];
  const bool cin = kf != invalid && prevk == kf;
  const bool cout = kl != invalid && nextk == kl;
  float* part = d.part + (int64_t)blockIdx.x * 2 * 32 + ch;
  // the run continuing from the previous chunk: its pieces here, summed by half-wave 0
  if (hw == 0 && cin) {
    float acc = racc[0][0][ch];
    bool open = nr == 1 && cout;
    for (int t = 1; open && t < 8; ++t) {
      acc = acc + racc[t][0][ch];
      open = rcnt[t] == 1 && rnext[t] == kf;
    }
    part[0] = acc;
  }
  // the last run starts here and goes on: its later pieces in this chunk added in order; it
  // is written below if it ends in the chunk (closed), else its piece goes to k_det_join
  bool closed = false;
  if (cout && !(nr == 1 && cin)) {
    float acc = racc[hw][nr - 1][ch];
    bool open = true;
    for (int t = hw + 1; open && t < 8; ++t) {
      acc = acc + racc[t][0][ch];
      open = rcnt[t] == 1 && rnext[t] == kl;
    }
    if (open) {
      part[(hw == 0 && nr == 1) ? 0 : 32] = acc;  // the chunk's first run (slot 0) or its last
    } else {
      racc[hw][nr - 1][ch] = acc;
      closed = true;
    }
  }
  const bool skip_first = cin, skip_last = cout && !closed;
  const DetRows R = det_rows(m);
  const uint64_t vmask = (uint64_t(1) << d.vbits) - 1;
  // the runs that lie inside the sub-chunk, RG at a time: the group's sparse row ids, then
  // its destination values, read with their loads in flight together, then added to and
  // stored -- one writer per voxel, no atomics.  (All 32 at once kept 32 pointers and
  // values live: the compiler put them in scratch, and every reload waited vmcnt(0).)
#ifndef NC_DET_RG
#define NC_DET_RG 8
#endif
  constexpr int RG = NC_DET_RG;
  for (int r0 = 0; r0 < nr; r0 += RG) {
    float* dst[RG];
    if (R.fast) {  // branch-free: the row ids and the destinations are selects
      int32_t row[RG];
#pragma unroll
      for (int u = 0; u < RG; ++u) {
        const int r = r0 + u < nr ? r0 + u : nr - 1;
        const K k = rkey[hw][r];
        const int j = (int)((uint64_t)k >> d.vbits);
        const int32_t* rows = j == 0 ? R.rows[0] : j == 1 ? R.rows[1] : R.rows[2];
        // the invalid key (all ones: j = 3, voxel 2^vbits - 1) is in every sort's tail; its
        // voxel index lies at or past the end of job 2's [D*H*W] row map, so it reads val[0]
        const bool live = rows != nullptr && k != invalid;
        row[u] = R.any_rows ? *(live ? rows + ((uint64_t)k & vmask) : reinterpret_cast<const int32_t*>(val)) : 0;
      }
#pragma unroll
      for (int u = 0; u < RG; ++u) {
        const int r = r0 + u < nr ? r0 + u : nr - 1;
        const K k = rkey[hw][r];
        const int j = (int)((uint64_t)k >> d.vbits);
        const int32_t* rows = j == 0 ? R.rows[0] : j == 1 ? R.rows[1] : R.rows[2];
        float* g = j == 0 ? R.grad[0] : j == 1 ? R.grad[1] : R.grad[2];
        const int64_t rr = rows ? (int64_t)row[u] : (int64_t)((uint64_t)k & vmask);
        const bool ok = r0 + u < nr && k != invalid && !(r == 0 && skip_first) && !(r == nr - 1 && skip_last) &&
                        rr >= 0;
        dst[u] = ok ? g + rr * 32 + ch : nullptr;
      }
    } else {  // a strided dense gradient
#pragma unroll
      for (int u = 0; u < RG; ++u) {
        const int r = r0 + u < nr ? r0 + u : nr - 1;
        const K k = rkey[hw][r];
        const bool ok = r0 + u < nr && k != invalid && !(r == 0 && skip_first) && !(r == nr - 1 && skip_last);
        dst[u] = ok ? det_dst(m, d, (uint64_t)k, ch) : nullptr;
      }
    }
    float old[RG];
#pragma unroll
    for (int u = 0; u < RG; ++u) old[u] = *(dst[u] ? dst[u] : d.w);  // d.w[0] when nothing is written
#pragma unroll
    for (int u = 0; u < RG; ++u) {
      const int r = r0 + u;
      if (r >= nr) break;
      const K k = rkey[hw][r];
      if (k == invalid) continue;
      const float a = racc[hw][r][ch];
      if (dst[u]) *dst[u] = old[u] + a;
    }
  }
}

// half-wave = chunk s (DCH entries): if a run starts in s and continues past it, sum its
// pieces.  The four neighbour keys are read together and the following chunks' pieces and
// end keys JOIN_AHEAD at a time (clamped, unconditional loads); the pieces are still added
// one by one in chunk order
constexpr int JOIN_AHEAD = 4;
template <typename K>
__global__ void __launch_bounds__(256) k_det_join(const MlpCtx m, DetBufs d, int64_t n) {
  const int64_t s = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int ch = threadIdx.x & 31;
  const int64_t e0 = s * DCH;
  if (e0 >= n) return;
  const int64_t e1 = e0 + DCH < n ? e0 + DCH : n;
  const int64_t nsub = (n + DCH - 1) / DCH;
  const K* key = reinterpret_cast<const K*>(d.sorted ? d.key[1] : d.key[0]);  // select: a runtime index into the argument copies it to scratch
  const K invalid = (K)((uint64_t(1) << (d.vbits + 2)) - 1);
  const K last = key[e1 - 1];
  const K after = key[e1 < n ? e1 : e1 - 1];
  const K first = key[e0];
  const K before = key[e0 > 0 ? e0 - 1 : e0];
  // (non-short-circuit: all four loads are used before the one exit, so none is sunk past it)
  const bool cont = (last != invalid) & (e1 < n) & (after == last);  // a run continues past s
  const bool single = first == last;
  if (!(cont & !(single & (e0 > 0) & (before == last)))) return;  // or it started before s: not the owner
  float acc = d.part[(s * 2 + (single ? 0 : 1)) * 32 + ch];
  for (int64_t t = s + 1;; t += JOIN_AHEAD) {
    float pv[JOIN_AHEAD];
    K kv[JOIN_AHEAD];
#pragma unroll
    for (int u = 0; u < JOIN_AHEAD; ++u) {
      const int64_t tt = t + u < nsub ? t + u : nsub - 1;
      const int64_t te = (tt + 1) * DCH;
      pv[u] = d.part[tt * 2 * 32 + ch];
      kv[u] = key[te < n ? te : n - 1];
    }
    bool done = false;
#pragma unroll
    for (int u = 0; u < JOIN_AHEAD; ++u) {
      if (!done) {
        acc = acc + pv[u];
        const int64_t te = (t + u + 1) * DCH;
        done = te >= n || kv[u] != last;  // the run ends inside t + u (or at its end)
      }
    }
    if (done) break;
  }
  const DetRows R = det_rows(m);
  float* dst;
  if (R.fast) {
    const int j = (int)((uint64_t)last >> d.vbits);
    const uint64_t v = (uint64_t)last & ((uint64_t(1) << d.vbits) - 1);
    const int32_t* rows = j == 0 ? R.rows[0] : j == 1 ? R.rows[1] : R.rows[2];
    float* g = j == 0 ? R.grad[0] : j == 1 ? R.grad[1] : R.grad[2];
    const int64_t rr = rows ? (int64_t)rows[v] : (int64_t)v;
    dst = rr >= 0 ? g + rr * 32 + ch : nullptr;
  } else {
    dst = det_dst(m, d, (uint64_t)last, ch);
  }
  if (dst) *dst = *dst + acc;
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort of (key, entry id), RS_BITS per pass, for the deterministic
// scatter.  Reduce-then-scan: every pass is three plain kernels whose state is entirely
// rewritten by the pass itself -- no memsets, no counters carried between launches, no
// workgroup waiting on another (a hipGraph replays it like any other kernel chain).
// This replaces rocprim's radix sort here: its onesweep path (taken above 1M items)
// resets a decoupled look-back state and an atomic block-id counter with two
// hipMemsetAsync per digit pass and then spins on other workgroups' flags; in the
// captured graph those resets are memset nodes, and a look-back state not yet zeroed
// when the pass starts reads as a predecessor's COMPLETE prefix of the previous pass or
// replay (scatter offsets off -> entry ids never written -> the faulting gather that was
// seen) or a stale block id whose predecessor never publishes (the look-back spin that
// was seen).  Both recorded failures are that one mechanism; the sort below has none of
// it: it is capture-safe by construction, and faster at these sizes.
//   k_rs_hist     tile of RS_TILE keys per workgroup -> its digit counts, tile-major
//                 hist[tile][d] (one coalesced row per tile; digit-major rows were 4-byte
//                 writes a tile apart)
//   k_rs_scan     RS_SCAN_DIG digits per workgroup: exclusive scan of hist[*][d] over the
//                 tiles in place, total[d]
//   k_rs_scatter  tile rank by rank: 256 entries per round in input order, stable rank
//                 inside the wave from 8 ballots, wave offsets through LDS; destination =
//                 exclusive scan of total[] + hist[tile][d] + rank so far
// ---------------------------------------------------------------------------

template <int BITS, typename K>
__device__ __forceinline__ int rs_digit(K k, int bit) {
  return (int)((k >> bit) & (K)((1 << BITS) - 1));
}

template <int BITS, typename K>
__global__ void __launch_bounds__(RS_THREADS) k_rs_hist(const K* __restrict__ key, int64_t n, int bit,
                                                        uint32_t* __restrict__ hist, int64_t ntile) {
  constexpr int BINS = 1 << BITS;
  __shared__ uint32_t cnt[BINS];
  for (int b = threadIdx.x; b < BINS; b += RS_THREADS) cnt[b] = 0u;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
#pragma unroll 4
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int64_t e = base + r * RS_THREADS + threadIdx.x;
    if (e < n) atomicAdd(&cnt[rs_digit<BITS>(key[e], bit)], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < BINS; b += RS_THREADS) hist[(int64_t)blockIdx.x * BINS + b] = cnt[b];
}

// block-wide exclusive scan of one value per thread (RS_THREADS = 4 waves); returns the
// block total through *total
__device__ __forceinline__ uint32_t rs_block_exscan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int q = 0; q < RS_THREADS / 64; ++q) {
    before += q < w ? wsum[q] : 0u;
    all += wsum[q];
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

// tile-major counts hist[tile][digit] (the per-tile writes and reads are whole rows): a
// workgroup scans RS_SCAN_DIG digits, its threads in RS_THREADS / RS_SCAN_DIG groups of
// consecutive tiles -- the group sums, their exclusive prefix through LDS, then the
// in-place exclusive scan of each group's range
#ifndef NC_RS_SCAN_DIG
#define NC_RS_SCAN_DIG 16
#endif
constexpr int RS_SCAN_DIG = NC_RS_SCAN_DIG;
constexpr int RS_SCAN_REG = 48;  // tiles per thread held in registers (C2: 36); more: two passes over memory
template <int BITS>
__global__ void __launch_bounds__(RS_THREADS) k_rs_scan(uint32_t* __restrict__ hist, int64_t ntile,
                                                        uint32_t* __restrict__ total) {
  constexpr int BINS = 1 << BITS, TG = RS_THREADS / RS_SCAN_DIG;
  __shared__ uint32_t part[TG][RS_SCAN_DIG];
  const int dl = threadIdx.x % RS_SCAN_DIG, g = threadIdx.x / RS_SCAN_DIG;
  const int b = blockIdx.x * RS_SCAN_DIG + dl;
  const int64_t per = (ntile + TG - 1) / TG;
  const int64_t t0 = g * per < ntile ? g * per : ntile, t1 = t0 + per < ntile ? t0 + per : ntile;
  uint32_t sum = 0;
  if (per <= RS_SCAN_REG) {  // the group's counts held in registers between the two passes,
    uint32_t cv[RS_SCAN_REG];  // loaded together (clamped, unconditional)
#pragma unroll
    for (int i = 0; i < RS_SCAN_REG; ++i) {
      const int64_t t = t0 + i < t1 ? t0 + i : (t1 > 0 ? t1 - 1 : 0);
      cv[i] = hist[t * BINS + b];
    }
#pragma unroll
    for (int i = 0; i < RS_SCAN_REG; ++i) sum += t0 + i < t1 ? cv[i] : 0u;
    part[g][dl] = sum;
    __syncthreads();
    uint32_t run = 0, all = 0;
#pragma unroll
    for (int q = 0; q < TG; ++q) {
      run += q < g ? part[q][dl] : 0u;
      all += part[q][dl];
    }
#pragma unroll
    for (int i = 0; i < RS_SCAN_REG; ++i) {
      if (t0 + i < t1) hist[(t0 + i) * BINS + b] = run;
      run += t0 + i < t1 ? cv[i] : 0u;
    }
    if (g == 0) total[b] = all;
    return;
  }
#pragma unroll 8
  for (int64_t t = t0; t < t1; ++t) sum += hist[t * BINS + b];
  part[g][dl] = sum;
  __syncthreads();
  uint32_t run = 0, all = 0;
#pragma unroll
  for (int q = 0; q < TG; ++q) {
    run += q < g ? part[q][dl] : 0u;
    all += part[q][dl];
  }
#pragma unroll 8
  for (int64_t t = t0; t < t1; ++t) {
    const uint32_t c = hist[t * BINS + b];
    hist[t * BINS + b] = run;
    run += c;
  }
  if (g == 0) total[b] = all;
}

// BINS = 2^BITS digits, BPT = BINS / RS_THREADS of them per thread (consecutive)
template <int BITS, typename K>
__global__ void __launch_bounds__(RS_THREADS) k_rs_scatter(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                           K* __restrict__ kout, uint32_t* __restrict__ vout, int64_t n,
                                                           int bit, const uint32_t* __restrict__ hist, int64_t ntile,
                                                           const uint32_t* __restrict__ total) {
  constexpr int BINS = 1 << BITS, BPT = BINS / RS_THREADS;
  __shared__ uint32_t start[BINS];                 // next output slot of each digit for this tile
  __shared__ uint32_t wcnt[RS_THREADS / 64][BINS];  // this round's count of each digit per wave
  __shared__ uint32_t wsum[RS_THREADS / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  {
    uint32_t t[BPT], sum = 0;
#pragma unroll
    for (int q = 0; q < BPT; ++q) sum += (t[q] = total[threadIdx.x * BPT + q]);
    uint32_t all;
    uint32_t base = rs_block_exscan(sum, wsum, &all);
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
      const int b = threadIdx.x * BPT + q;
      start[b] = base + hist[(int64_t)blockIdx.x * BINS + b];
      base += t[q];
    }
  }
  const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int64_t tile0 = (int64_t)blockIdx.x * RS_TILE;
  // the whole tile's keys and ids loaded up front (clamped, all in flight together), the
  // rounds then run from registers
  K kt[RS_ROUNDS];
  uint32_t vt[RS_ROUNDS];
#pragma unroll
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int64_t e = tile0 + r * RS_THREADS + threadIdx.x;
    kt[r] = kin[e < n ? e : n - 1];
  }
  if (vin) {
#pragma unroll
    for (int r = 0; r < RS_ROUNDS; ++r) {
      const int64_t e = tile0 + r * RS_THREADS + threadIdx.x;
      vt[r] = vin[e < n ? e : n - 1];
    }
  } else {  // first pass: entry id = position
#pragma unroll
    for (int r = 0; r < RS_ROUNDS; ++r) vt[r] = (uint32_t)(tile0 + r * RS_THREADS + threadIdx.x);
  }
#pragma unroll
  for (int r = 0; r < RS_ROUNDS; ++r) {
    const int64_t e = tile0 + r * RS_THREADS + threadIdx.x;
    if (tile0 + r * RS_THREADS >= n) break;  // block-uniform
#pragma unroll
    for (int q = 0; q < RS_THREADS / 64; ++q)
#pragma unroll
      for (int c = 0; c < BPT; ++c) wcnt[q][c * RS_THREADS + threadIdx.x] = 0u;
    const bool ok = e < n;
    const K k = ok ? kt[r] : (K)0;
    const uint32_t v = ok ? vt[r] : 0u;
    const int d = rs_digit<BITS>(k, bit);
    // lanes of this wave holding the same digit (and a valid entry)
    uint64_t same = __ballot(ok);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
      const uint64_t m = __ballot((d >> b) & 1);
      same &= ((d >> b) & 1) ? m : ~m;
    }
    const uint32_t rank = (uint32_t)__popcll(same & below);
    __syncthreads();  // wcnt zeroed; start[] of the previous round updated
    if (ok && rank == 0) wcnt[w][d] = (uint32_t)__popcll(same);
    __syncthreads();
    if (ok) {
      uint32_t off = start[d] + rank;
#pragma unroll
      for (int q = 0; q < RS_THREADS / 64; ++q) off += q < w ? wcnt[q][d] : 0u;
      kout[off] = k;
      vout[off] = v;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < BPT; ++c) {
      const int b = c * RS_THREADS + threadIdx.x;
      uint32_t add = 0;
#pragma unroll
      for (int q = 0; q < RS_THREADS / 64; ++q) add += wcnt[q][b];
      start[b] += add;
    }
  }
}

static int64_t rs_tiles(int64_t n) { return (n + RS_TILE - 1) / RS_TILE; }

// digit width: the fewest passes over end_bit key bits (at most RS_MAX_BITS per pass), then
// the narrowest digit that keeps that count -- 20-bit keys (the C2 grids) sort in 2 passes
// of 10 bits instead of 3 of 8.  NC_DET_SORT_BITS=8..11 pins the width (read when the
// buffers are laid out; a stable sort has one result, so every width gives bit-identical
// gradients: test_gpu_determinism checks it)
int det_sort_bits(int end_bit) {
  const char* e = std::getenv("NC_DET_SORT_BITS");
  const int pinned = e ? std::atoi(e) : 0;
  if (pinned >= 8 && pinned <= RS_MAX_BITS) return pinned;
  const int passes = (end_bit + RS_MAX_BITS - 1) / RS_MAX_BITS;
  const int bits = (end_bit + passes - 1) / passes;
  return bits < 8 ? 8 : bits;
}

size_t det_sort_temp_bytes(int64_t n_entries, int bits) {
  const int64_t bins = int64_t(1) << bits;
  return (size_t)(bins * rs_tiles(n_entries) + bins) * 4;
}

// sorts key[0] (with the entry ids, taken from the positions by the first pass) by the low
// end_bit bits; returns the buffer index holding the result
// (the first pass's counts are k_det_keys' when its workgroups are the sort's tiles)
template <int BITS, typename K>
static int radix_sort_w(const DetBufs& d, int64_t n, int end_bit, hipStream_t s, int* sorted) {
  constexpr int BINS = 1 << BITS;
  const int64_t nt = rs_tiles(n);
  uint32_t* hist = reinterpret_cast<uint32_t*>(d.temp);
  uint32_t* total = hist + BINS * nt;
  int src = 0;
  for (int bit = 0; bit < end_bit; bit += BITS) {
    const K* kin = reinterpret_cast<const K*>(d.key[src]);
    K* kout = reinterpret_cast<K*>(d.key[1 - src]);
    if (bit > 0 || !KEYS_HIST)
      hipLaunchKernelGGL((k_rs_hist<BITS, K>), dim3((unsigned)nt), dim3(RS_THREADS), 0, s, kin, n, bit, hist, nt);
    hipLaunchKernelGGL(k_rs_scan<BITS>, dim3(BINS / RS_SCAN_DIG), dim3(RS_THREADS), 0, s, hist, nt, total);
    hipLaunchKernelGGL((k_rs_scatter<BITS, K>), dim3((unsigned)nt), dim3(RS_THREADS), 0, s, kin,
                       bit == 0 ? (const uint32_t*)nullptr : d.val[src], kout,
                       d.val[1 - src], n, bit, hist, nt, total);
    if (hipError_t e = hipGetLastError()) return (int)e;
    src = 1 - src;
  }
  *sorted = src;
  return 0;
}

template <typename K>
static int radix_sort(const DetBufs& d, int64_t n, int end_bit, hipStream_t s, int* sorted) {
  switch (d.sort_bits) {
    case 8: return radix_sort_w<8, K>(d, n, end_bit, s, sorted);
    case 9: return radix_sort_w<9, K>(d, n, end_bit, s, sorted);
    case 10: return radix_sort_w<10, K>(d, n, end_bit, s, sorted);
    case 11: return radix_sort_w<11, K>(d, n, end_bit, s, sorted);
    default: return (int)hipErrorInvalidValue;
  }
}

template <typename K>
static int det_scatter(const MlpCtx& m, const DetBufs& d0, int64_t n, hipStream_t s) {
  DetBufs d = d0;
  // workspace first: k_det_keys already writes the first pass's tile counts into d.temp
  if (d.temp_bytes < det_sort_temp_bytes(n, d.sort_bits)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_det_keys<K>, dim3((unsigned)(d.ppad / DET_TILE_POINTS), m.n_jobs), dim3(DET_TILE_POINTS), 0, s,
                     m, d);
  if (hipError_t e = hipGetLastError()) return (int)e;
  if (int e = radix_sort<K>(d, n, d.vbits + 2, s, &d.sorted)) return e;
  const int64_t nch = (n + DCH - 1) / DCH;  // chunks = k_det_runs workgroups
  hipLaunchKernelGGL(k_det_runs<K>, dim3((unsigned)nch), dim3(256), 0, s, m, d, n);
  if (hipError_t e = hipGetLastError()) return (int)e;
  hipLaunchKernelGGL(k_det_join<K>, dim3((unsigned)((nch + 7) / 8)), dim3(256), 0, s, m, d, n);
  return (int)hipGetLastError();
}

int launch_det_scatter(const MlpCtx& m, const DetBufs& d, hipStream_t s) {
  const int64_t n = (int64_t)m.n_jobs * d.ppad * 8;  // entries, each job's points padded (k_det_keys)
  if (m.P == 0 || n == 0) return 0;
  if (d.ppad != det_ppad(m.P)) return (int)hipErrorInvalidValue;
  return d.vbits + 2 <= 32 ? det_scatter<uint32_t>(m, d, n, s) : det_scatter<uint64_t>(m, d, n, s);
}

}  // namespace nc
