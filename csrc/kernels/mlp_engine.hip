// Persistent decode post-attention tail for batch 1 on gfx950 (the loader-ring engine):
//     h += bf16(sum_s P[s]);  x = rmsnorm(h) * gamma        (P: the o_proj split-K slabs; or x given)
//     h += W_down . (silu(W_gate . x) * (W_up . x))
// as ONE launch of one workgroup per CU, instead of add_partials_rmsnorm + the SiLU*up stream GEMM +
// the down GEMM (three launches, two of them with their own grid fill and drain around a 235 / 117 MB
// weight stream). Measured (Llama-3.1-8B shapes, hipGraph replay, profiles/mlp_engine_r5.log): 64 vs
// 70 us per layer; batch-1 decode step 3.44-3.47 -> 3.33 ms.
//
// Why: at batch 1 the decode layer is a weight stream, and each launch boundary costs the stream a
// fill (the first loads of every block start cold) and a drain (the tail of the slowest blocks).
// Here the weights of BOTH projections go through one LDS ring per CU without a break: the ring's
// loader does not depend on the activations, so while the consumers wait for the chip-wide
// hand-off between the two projections (every CU needs all I activations before it can start the
// down projection), the loader is already filling the ring with down-projection weights.
//
// Workgroup = 4 waves: wave 0 = loader, waves 1..3 = consumers (ME_NLOAD / ME_THREADS: one loader wave
// measured the same as two -- the HBM stream, not the in-flight depth, is the limit).
//   * work split: workgroup w owns 8-wide groups of activations [a0, a1) (gate rows and up rows of
//     those activations from the packed [64 gate | 64 up] weight tiles) and 16-row groups of output
//     rows [d0, d1) of the down projection; a ring slot = 16 weight rows x 512 K columns (16 KiB):
//     phase A slots (8 gate + 8 up rows, chunk fastest), then phase B slots (16 down rows);
//   * loader: LDS-DMA (global_load_lds, 16 B per lane, one instruction per 1 KiB row piece), up to
//     ME_INFLIGHT slots in flight, a slot published (LDS word FULL = seq + 1) behind a counted vmcnt;
//     a slot is refilled only after its consumer wrote FREE = seq + 1 (after its fragment reads);
//   * consumers: slot s goes to consumer s % 3; its 16 rows are one MFMA 16x16x32 column tile
//     (x broadcast in the A operand: row m = 0 of the product is the result), 16 K-steps per slot;
//     the 16 per-slot sums go to an LDS partial array (summed in a fixed order later: deterministic);
//   * end of phase A (the last consumer to arrive, LDS counter): act = bf16(silu(gate) * up) for the
//     workgroup's activations, stored write-through (sc1, 8-B agent stores) to the act workspace,
//     vmcnt(0), then ONE agent-scope atomic add on this workgroup's counter shard (8 shards, one per
//     XCD in dispatch order; a shard's last arriver adds to a top counter); one lane polls the top
//     counter (sc1 loads) until every workgroup of this launch arrived, then the wave loads all I
//     activations with sc1 buffer loads into LDS and sets an LDS word the other consumers wait on;
//   * fused tail (P given): before phase A every workgroup forms the whole row h + bf16(sum P) and its
//     norm (add_partials_rmsnorm's math) from the slabs while the loader's first slots are in flight;
//     it keeps its own down rows of that residual and writes h only at its end;
//   * end of phase B (last consumer): h[row] = bf16(h[row] + sum of the row's partials).
// Counters are monotonic (never re-zeroed between launches, so a hipGraph replay needs no memset
// node): a workgroup's own add returns the count before it, which names the launch generation; the
// shard's last arriver adds to the top counter, which the waiters poll for (generation + 1) x shards.
// Every wait is bounded by ONE deadline per workgroup (s_memrealtime at entry + the timeout word, 100 ms by
// default): a wait that gives up writes the error code to the device error word AND to a host-mapped
// pinned word, raises this workgroup's LDS abort flag (every other wave of the workgroup leaves its own
// wait at its next check), and the workgroup then writes NOTHING: no h rows, no activations past the
// failure, no slots published that were never loaded. A launch that finds the device error word already
// set (an earlier launch of the same step failed) exits before touching any state, so the step's later
// layers cannot mis-synchronise on counters the failed launch left off their generation. The engine reads
// the host word after every decode step's existing event sync (no extra device sync), discards that step
// and the one in flight behind it, re-arms the counters and recomputes them on the separate kernels
// (engine/llm_engine.py _recover_engine_fault).
// Deadlock freedom: one workgroup per CU (the LDS footprint admits one), grid = CU count, all
// resident; the only cross-workgroup wait is the act hand-off. (A GPU shared with another process's
// long-running kernels can keep a workgroup from being dispatched: the bounded wait then reports a
// timeout instead of hanging; the model uses the engine only at TP = 1.)
#include "common.h"
#include <cstring>
using namespace ragk;

namespace {

constexpr int ME_THREADS = 256;
constexpr int ME_ROWS = 16;                        // weight rows per slot
constexpr int ME_KC = 512;                         // K columns per slot
constexpr int ME_PITCH = ME_KC * 2 + 16;           // LDS row pitch: 16-B skew between consecutive rows
constexpr int ME_SLOT = ME_ROWS * ME_PITCH;        // 16640 B
constexpr int ME_RING = 7;
constexpr int ME_INFLIGHT = 3;                     // slots in flight behind the newest issue
constexpr int ME_NLOAD = 1;                       // loader waves (slot s: loader s % ME_NLOAD)
constexpr int ME_NCONS = ME_THREADS / 64 - ME_NLOAD;  // consumer waves
constexpr int ME_VEC = 28672;                      // x (phase A) / act (phase B) bytes: max(2H, 2I)
constexpr int ME_MAXA = 64, ME_MAXB = 56;          // slots per workgroup and phase
constexpr int ME_SHARDS = 8;
constexpr int ME_CTR_STRIDE = 16;                  // u64 per shard: one 128-B line each
constexpr unsigned ME_TIMEOUT_TICKS = 10000000u;   // default deadline: 100 ms of s_memrealtime (100 MHz)
// error codes (device word, host word): which wait gave up
constexpr unsigned ME_ERR_HANDOFF = 1u, ME_ERR_SLOT = 2u, ME_ERR_FREE = 3u, ME_ERR_ACT = 4u;

struct MlpArgs {
  const bf16_t* xn;        // [H] normalised input row (P == nullptr)
  const float* P;          // [S][H] o_proj split-K slabs: h += bf16(sum P), x = rmsnorm(h) * gamma in-launch
  const bf16_t* gamma;     // [H] post-attention norm weight (with P)
  float eps;
  int S;
  const bf16_t* wgu;       // [2I][H] packed [64 gate | 64 up] per 128 rows
  const bf16_t* wd;        // [H][I]
  bf16_t* h;               // [H] residual, updated in place
  bf16_t* act;             // [I] hand-off workspace
  unsigned long long* ctr; // [ME_SHARDS][ME_CTR_STRIDE] arrival counters
  unsigned* err;           // device error word (0 = healthy); a set word makes later launches exit at entry
  unsigned* err_host;      // device address of a host-mapped pinned word (the engine polls it per step)
  const unsigned* tmo;     // deadline in s_memrealtime ticks (0 = ME_TIMEOUT_TICKS); a test hook forces timeouts
  unsigned long long* stamps;  // optional [G][8] s_memrealtime stamps (tools/mlp_engine_bench.py ME_STAMPS=1)
  int H, I;
  int w_even, w_odd;       // phase-A work weights of workgroups on even / odd XCDs
};

// prefix weight of workgroups [0, w): even w weigh we, odd wo
__host__ __device__ __forceinline__ long long me_cum(int w, int we, int wo) {
  return (long long)(w / 2) * (we + wo) + (long long)(w & 1) * we;
}

// Workgroup w's share: activation groups [r[0], r[1]) (weighted by XCD parity), down row groups [r[2], r[3])
__host__ __device__ __forceinline__ void me_split(int G, int w, int NA, int ND, int we, int wo, int (&r)[4]) {
  const long long T = me_cum(G, we, wo);
  r[0] = (int)((long long)NA * me_cum(w, we, wo) / T);
  r[1] = (int)((long long)NA * me_cum(w + 1, we, wo) / T);
  r[2] = (int)((long long)w * ND / G);
  r[3] = (int)((long long)(w + 1) * ND / G);
}

__device__ __forceinline__ void me_stamp(const MlpArgs& a, int i) {
  if (a.stamps) a.stamps[blockIdx.x * 8 + i] = __builtin_amdgcn_s_memrealtime();
}

struct MlpSmem {
  char ring[ME_RING * ME_SLOT];
  char vec[ME_VEC];
  float part[(ME_MAXA + ME_MAXB) * ME_ROWS];
  bf16_t actl[64];
  float hres[64];          // this workgroup's rows of h after the o_proj residual (fused tail)
  float red[8];
  unsigned full[8], freew[8];
  unsigned doneA, doneB, actReady, abort;
};

__device__ __forceinline__ void unpack4(uint2 v, float (&f)[4]) {
  f[0] = __uint_as_float(v.x << 16);
  f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16);
  f[3] = __uint_as_float(v.y & 0xffff0000u);
}

template <int N>
__device__ __forceinline__ void me_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (((N >> 4) & 3) << 14) | (0x7 << 4) | (0xF << 8));
}
__device__ __forceinline__ void me_wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// LDS flag words: explicit address-space-3 volatile accesses (a generic volatile pointer compiles to
// flat_load / flat_store, which also count in vmcnt and would break the loader's counted waits)
typedef __attribute__((address_space(3))) volatile unsigned lds_u32;
__device__ __forceinline__ unsigned lds_ld(const unsigned* p) { return *(const lds_u32*)(p); }
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) { *(lds_u32*)(p) = v; }

__device__ __forceinline__ unsigned long long me_now() { return __builtin_amdgcn_s_memrealtime(); }

// A wait gave up: report (device word for the launches behind this one, host word for the engine) and
// raise the workgroup's abort flag.
__device__ __forceinline__ void me_fail(const MlpArgs& a, MlpSmem& sm, unsigned code) {
  __hip_atomic_store(a.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.err_host) __hip_atomic_store(a.err_host, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  lds_st(&sm.abort, 1u);
}

// bounded spin on an LDS word (same workgroup): true when *p == want; false when this workgroup aborted
// (another wave gave up) or the deadline passed (this wave gives up)
__device__ __forceinline__ bool me_spin_lds(const unsigned* p, unsigned want, const MlpArgs& a, MlpSmem& sm,
                                            unsigned long long deadline, unsigned code) {
  for (unsigned it = 0; lds_ld(p) != want; ++it) {
    if ((it & 31) == 31) {
      if (lds_ld(&sm.abort)) return false;
      if (me_now() > deadline) {
        me_fail(a, sm, code);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

struct SlotMap {
  int a0, nA, d0, KA, KB;
  __device__ __forceinline__ int chunk(int s) const { return s < nA ? s % KA : (s - nA) % KB; }
};

// The loader's wave-uniform cursor over its slots (no divisions in the issue loop): slot s, group g
// (activation group in phase A, down row group in phase B), K chunk kc; the slot's 16 rows are
// base + r * stride (+ jump for the up rows: packed row of up j = packed row of gate j + 64).
struct LoadCursor {
  int s = 0, g = 0, kc = 0;
  __device__ __forceinline__ void next(const SlotMap& m) {
    ++s;
    ++kc;
    if (s == m.nA) {
      g = 0;
      kc = 0;
    } else if (kc == (s < m.nA ? m.KA : m.KB)) {
      kc = 0;
      ++g;
    }
  }
};

template <bool NT>
__device__ __forceinline__ void me_issue_slot(const MlpArgs& a, const SlotMap& m, const LoadCursor& cu, MlpSmem& sm,
                                              int lane) {
  char* dst = sm.ring + (cu.s % ME_RING) * ME_SLOT;
  const char* base;
  long long stride, jump;
  if (cu.s < m.nA) {
    const int j0 = 8 * (m.a0 + cu.g);
    const int prow0 = (j0 >> 6) * 128 + (j0 & 63);
    base = reinterpret_cast<const char*>(a.wgu) + (long long)prow0 * a.H * 2 + cu.kc * (ME_KC * 2);
    stride = 2ll * a.H;
    jump = 112ll * a.H;
  } else {
    base = reinterpret_cast<const char*>(a.wd) + (long long)(16 * (m.d0 + cu.g)) * a.I * 2 + cu.kc * (ME_KC * 2);
    stride = 2ll * a.I;
    jump = 0;
  }
#pragma unroll
  for (int r = 0; r < ME_ROWS; ++r) {
    const char* src = base + r * stride + (r >= 8 ? jump : 0) + lane * 16;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(dst + r * ME_PITCH), 16, 0,
                                     NT ? 2 : 0);
  }
}

template <bool NT>
__global__ __launch_bounds__(ME_THREADS, 1) void mlp_engine_kernel(MlpArgs a) {
  __shared__ __attribute__((aligned(16))) MlpSmem sm;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int G = gridDim.x, w = blockIdx.x;
  const int NA = a.I / 8, ND = a.H / 16;
  SlotMap m;
  m.KA = a.H / ME_KC;
  m.KB = a.I / ME_KC;
  // activation groups split in proportion to per-XCD stream rate (dispatch order w % 8 = XCD): the
  // workgroups on even XCDs streamed the same phase-A work ~15 % slower, repeatably (correlation 0.97
  // launch to launch, profiles/mlp_engine_skew_r5.log), and the hand-off waits for the slowest
  int rng[4];
  me_split(G, w, NA, ND, a.w_even, a.w_odd, rng);
  m.a0 = rng[0];
  const int a1 = rng[1];
  m.d0 = rng[2];
  const int d1 = rng[3];
  m.nA = (a1 - m.a0) * m.KA;
  const int nB = (d1 - m.d0) * m.KB;
  const int nS = m.nA + nB;
  // this workgroup's deadline for every wait below (one clock, one bound)
  const unsigned tk = *a.tmo;
  const unsigned long long deadline = me_now() + (tk ? tk : ME_TIMEOUT_TICKS);

  if (wid < ME_NLOAD) {
    if (wid == 0) {
      if (lane == 0) me_stamp(a, 0);
      if (lane < 8) {
        sm.full[lane] = 0u;
        sm.freew[lane] = 0u;
      }
      if (lane == 0) {
        sm.doneA = 0u;
        sm.doneB = 0u;
        sm.actReady = 0u;
        // an earlier launch failed (its workgroups left the counters off their generation): skip
        sm.abort = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 1u : 0u;
      }
    }
    // each loader's first ME_INFLIGHT slots (ME_NLOAD x ME_INFLIGHT < ME_RING: no slot is reused yet)
    LoadCursor cu;
    for (int k = 0; k < wid; ++k) cu.next(m);
    for (int k = 0; k < ME_INFLIGHT && cu.s < nS; ++k) {
      me_issue_slot<NT>(a, m, cu, sm, lane);
      for (int q = 0; q < ME_NLOAD; ++q) cu.next(m);
    }
  } else if (!a.P) {
    // x -> LDS (written by the previous launch: plain loads)
    const int t = threadIdx.x - 64 * ME_NLOAD;
    for (int i = t; i < a.H / 8; i += ME_THREADS - 64 * ME_NLOAD)
      *reinterpret_cast<u32x4*>(sm.vec + 16 * i) = *reinterpret_cast<const u32x4*>(a.xn + 8 * i);
  }
  if (a.P) {
    // fused post-attention tail (all waves; the loader has its first slots in flight), pass 1:
    // hn = bf16(h + bf16(sum_s P[s])) -> LDS, sum of squares (add_partials_rmsnorm's math). Every
    // workgroup forms the whole row (the norm needs all of it); it keeps its own down rows of hn for
    // the final residual and writes h only at its end (every reader of h is past its phase A by then).
    const int t = threadIdx.x;
    float ss = 0.f;
    const int n4 = a.H / 4;
    constexpr int U = 2;
    constexpr int CT = ME_THREADS;
    for (int i0 = 0; i0 < n4; i0 += U * CT) {
      f32x4 pv[U][8];
      uint2 hv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = min(i0 + u * CT + t, n4 - 1);
#pragma unroll
        for (int s = 0; s < 8; ++s)
          if (s < a.S) pv[u][s] = *reinterpret_cast<const f32x4*>(a.P + (size_t)s * a.H + 4 * i);
        hv[u] = *reinterpret_cast<const uint2*>(a.h + 4 * i);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * CT + t;
        if (i >= n4) continue;
        f32x4 acc = pv[u][0];
#pragma unroll
        for (int s = 1; s < 8; ++s)
          if (s < a.S) acc += pv[u][s];
        for (int s = 8; s < a.S; ++s) acc += *reinterpret_cast<const f32x4*>(a.P + (size_t)s * a.H + 4 * i);
        float hf[4];
        unpack4(hv[u], hf);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = bf2f(f2bf(hf[e] + bf2f(f2bf(acc[e]))));
          ss += v[e] * v[e];
        }
        *reinterpret_cast<uint2*>(sm.vec + 8 * i) = make_uint2(pk2bf(v[0], v[1]), pk2bf(v[2], v[3]));
        const int r0 = 4 * i - 16 * m.d0;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (r0 + e >= 0 && r0 + e < 16 * (d1 - m.d0)) sm.hres[r0 + e] = v[e];
      }
    }
    ss = wave_sum(ss);
    if (lane == 0) sm.red[wid] = ss;
    me_wait_lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // pass 2, in place: x = bf16(gamma * bf16(hn * inv))
    float ssum = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < ME_THREADS / 64; ++w2) ssum += sm.red[w2];
    const float inv = rsqrtf(ssum / (float)a.H + a.eps);
    for (int i = t; i < n4; i += CT) {
      float hf[4], g[4], o[4];
      unpack4(*reinterpret_cast<const uint2*>(sm.vec + 8 * i), hf);
      unpack4(*reinterpret_cast<const uint2*>(a.gamma + 4 * i), g);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = g[e] * bf2f(f2bf(hf[e] * inv));
      *reinterpret_cast<uint2*>(sm.vec + 8 * i) = make_uint2(pk2bf(o[0], o[1]), pk2bf(o[2], o[3]));
    }
  }
  me_wait_lgkm0();
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (lds_ld(&sm.abort)) {  // skipped launch: touch nothing (drain the loader's first slots first)
    if (wid < ME_NLOAD) me_wait_vm<0>();
    return;
  }

  if (wid < ME_NLOAD) {
    // ---------------- loaders: slots wid, wid + ME_NLOAD, ... ----------------
    static_assert(ME_NLOAD * ME_INFLIGHT < ME_RING, "pre-issued slots must not wrap the ring");
    int pub = wid;  // oldest issued, unpublished slot of this loader
    bool ok = true;
    LoadCursor cu;
    for (int k = 0; k < wid + ME_NLOAD * ME_INFLIGHT; ++k) cu.next(m);
    for (; cu.s < nS;) {
      const int s = cu.s;
      const int r = s % ME_RING;
      if (s >= ME_RING) {
        const unsigned need = (unsigned)(s - ME_RING + 1);
        if (lds_ld(&sm.freew[r]) != need) {
          // the ring is full: publish what has landed before blocking on the consumers
          me_wait_vm<0>();
          for (; pub < s; pub += ME_NLOAD) lds_st(&sm.full[pub % ME_RING], (unsigned)pub + 1u);
          if (!me_spin_lds(&sm.freew[r], need, a, sm, deadline, ME_ERR_FREE)) {
            ok = false;  // aborted: issued slots past `pub` are never published
            break;
          }
        }
      }
      me_issue_slot<NT>(a, m, cu, sm, lane);
      if ((s - pub) / ME_NLOAD + 1 > ME_INFLIGHT) {
        me_wait_vm<16 * ME_INFLIGHT>();
        lds_st(&sm.full[pub % ME_RING], (unsigned)pub + 1u);
        pub += ME_NLOAD;
      }
      for (int q = 0; q < ME_NLOAD; ++q) cu.next(m);
    }
    if (lane == 0 && wid == 0) me_stamp(a, 1);
    me_wait_vm<0>();
    if (ok)
      for (; pub < nS; pub += ME_NLOAD) lds_st(&sm.full[pub % ME_RING], (unsigned)pub + 1u);
    return;
  }

  // ---------------- consumers ----------------
  const int c = wid - ME_NLOAD;
  const int n = lane & 15, kg = lane >> 4;
  bool arrivedA = false;
  // false: this workgroup aborted (or the hand-off timed out): the caller leaves without writing anything
  auto finish_A = [&]() -> bool {
    // called once per consumer, after its last phase-A slot (its partial stores retired)
    me_wait_lgkm0();
    if (lds_ld(&sm.abort)) return false;
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add(&sm.doneA, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    prev = __shfl(prev, 0, 64);
    if (prev != ME_NCONS - 1) return true;
    // last consumer of phase A: this workgroup's activations
    if (lane == 0) me_stamp(a, 2);
    const int nact = m.nA / m.KA * 8;  // <= 64
    if (lane < nact) {
      const int g = lane >> 3, jj = lane & 7;
      float gs = 0.f, us = 0.f;
      for (int kc = 0; kc < m.KA; ++kc) {
        const float* p = sm.part + (g * m.KA + kc) * ME_ROWS;
        gs += p[jj];
        us += p[8 + jj];
      }
      sm.actl[lane] = f2bf(silu(gs) * us);
    }
    me_wait_lgkm0();
    if (lane < nact / 4) {
      const unsigned long long v = *reinterpret_cast<const unsigned long long*>(sm.actl + 4 * lane);
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.act + 8 * m.a0 + 4 * lane), v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // arrive on this workgroup's shard; the count before the add names this launch's generation. The
    // last arriver of a shard adds to the top counter; the waiters poll only the top counter (one
    // load per poll: 256 workgroups polling 8 shard lines was ~38 G polls/s of fabric traffic beside
    // the other CUs' weight streams)
    const int shard = w & (ME_SHARDS - 1);
    const int nsh = G < ME_SHARDS ? G : ME_SHARDS;
    unsigned long long* top = a.ctr + ME_SHARDS * ME_CTR_STRIDE;
    unsigned long long want = 0;
    int failed = 0;
    if (lane == 0) {
      const unsigned long long mine = (unsigned long long)((G - shard + ME_SHARDS - 1) / ME_SHARDS);
      const unsigned long long old =
          __hip_atomic_fetch_add(a.ctr + shard * ME_CTR_STRIDE, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long gen = old / mine;
      if (old + 1 == (gen + 1) * mine) __hip_atomic_fetch_add(top, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      want = (gen + 1) * (unsigned long long)nsh;
      while (__hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        if (me_now() > deadline) {  // another workgroup never arrived: no activations are read
          me_fail(a, sm, ME_ERR_HANDOFF);
          failed = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
    }
    if (__shfl(failed, 0, 64)) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the poll
    // all I activations -> LDS, every load sc1 (the producers stored them sc1)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.act, 0, a.I * 2, 0x00020000);
    // every load in flight at once (one round trip; 7 dependent groups of 4 cost ~5 us here)
    constexpr int NV = ME_VEC / 1024;
    const int nv = a.I / 8;
    u32x4 v[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = 64 * u + lane;
      v[u] = i < nv ? __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * i, 0, 16))
                    : (u32x4){0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int i = 64 * u + lane;
      if (i < nv) *reinterpret_cast<u32x4*>(sm.vec + 16 * i) = v[u];
    }
    me_wait_lgkm0();
    if (lane == 0) lds_st(&sm.actReady, 1u);
    if (lane == 0) me_stamp(a, 3);
    return true;
  };

  bool actOk = false;
  for (int s = c; s < nS; s += ME_NCONS) {
    if (s >= m.nA && !arrivedA) {
      arrivedA = true;
      if (!finish_A()) return;
    }
    if (s >= m.nA && !actOk) {
      if (!me_spin_lds(&sm.actReady, 1u, a, sm, deadline, ME_ERR_ACT)) return;
      actOk = true;
    }
    const int r = s % ME_RING;
    if (!me_spin_lds(&sm.full[r], (unsigned)s + 1u, a, sm, deadline, ME_ERR_SLOT)) return;
    const char* slot = sm.ring + r * ME_SLOT;
    const char* xv = sm.vec + m.chunk(s) * (ME_KC * 2);
    bf16x8 wf[16], xf[16];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      wf[ks] = *reinterpret_cast<const bf16x8*>(slot + n * ME_PITCH + (ks * 32 + kg * 8) * 2);
      xf[ks] = *reinterpret_cast<const bf16x8*>(xv + (ks * 32 + kg * 8) * 2);
    }
    me_wait_lgkm0();
    if (lane == 0) lds_st(&sm.freew[r], (unsigned)s + 1u);
    // four independent accumulation chains (one dependent chain of 16 MFMAs made the consumers, not
    // the weight stream, the pace of the ring)
    f32x4 acc4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc4[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
      acc4[ks & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[ks], wf[ks], acc4[ks & 3], 0, 0, 0);
    const f32x4 acc = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
    // C[m][n]: lane (n, kg) holds rows 4kg..4kg+3 of column n; row 0 (x) sits in lanes 0..15
    if (lane < 16) sm.part[s * ME_ROWS + n] = acc[0];
  }
  if (!arrivedA && !finish_A()) return;

  // ---------------- phase B tail: the last consumer finishes the rows ----------------
  me_wait_lgkm0();
  if (lds_ld(&sm.abort)) return;  // a wave of this workgroup gave up: h stays unwritten
  unsigned prev = 0;
  if (lane == 0) prev = __hip_atomic_fetch_add(&sm.doneB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  prev = __shfl(prev, 0, 64);
  if (prev != ME_NCONS - 1) return;
  if (lds_ld(&sm.abort)) return;
  const int nd = d1 - m.d0;
  if (lane < 16 * nd) {
    const int g = lane >> 4, rr = lane & 15;
    float acc = 0.f;
    for (int kc = 0; kc < m.KB; ++kc) acc += sm.part[(m.nA + g * m.KB + kc) * ME_ROWS + rr];
    const int row = 16 * (m.d0 + g) + rr;
    a.h[row] = f2bf(acc + (a.P ? sm.hres[16 * g + rr] : bf2f(a.h[row])));
  }
  if (lane == 0) me_stamp(a, 4);
}

int g_me_nt = 1;
// measured per-XCD rate ratio ~0.84; for Llama-3.1-8B on 256 CUs (7 groups per workgroup on average)
// 27 : 32 and 3 : 4 give the same integer split, 6 : 8 groups (profiles/mlp_engine_xcd_weights_r5.log)
int g_me_w_even = 3, g_me_w_odd = 4;
unsigned long long* g_me_stamps = nullptr;

}  // namespace

// Whether the engine takes this shape on a grid of G workgroups (G = CU count).
RAGK_API int ragk_mlp_engine_ok(int M, int H, int I, int G) {
  if (M != 1 || G < 1 || H <= 0 || I <= 0) return 0;
  if (H % ME_KC || I % ME_KC || I % 64 || H % 16) return 0;
  if (2 * H > ME_VEC || 2 * I > ME_VEC) return 0;
  const int NA = I / 8, ND = H / 16;
  const long long T = me_cum(G, g_me_w_even, g_me_w_odd);
  const int wmax = g_me_w_even > g_me_w_odd ? g_me_w_even : g_me_w_odd;
  const int maxA = (int)(((long long)NA * wmax + T - 1) / T), maxB = (ND + G - 1) / G;  // floor-difference bound
  if (maxA * (H / ME_KC) > ME_MAXA || maxB * (I / ME_KC) > ME_MAXB || maxA * 8 > 64 || maxB * 16 > 64) return 0;
  return 1;
}

// The kernel's work split for workgroup w of G (CPU-tested: every activation group and down row group
// owned exactly once, per-workgroup slot counts within the LDS partial capacity).
RAGK_API int ragk_mlp_engine_split(int G, int w, int H, int I, int* out4) {
  if (G < 1 || w < 0 || w >= G || !out4) return (int)hipErrorInvalidValue;
  int r[4];
  me_split(G, w, I / 8, H / 16, g_me_w_even, g_me_w_odd, r);
  for (int i = 0; i < 4; ++i) out4[i] = r[i];
  return 0;
}

// phase-A weights of workgroups on even / odd XCDs (A/B tooling: 1, 1 = the even split)
RAGK_API int ragk_mlp_engine_set_xcd_weights(int we, int wo) {
  if (we < 1 || wo < 1 || we > 1000 || wo > 1000) return (int)hipErrorInvalidValue;
  g_me_w_even = we;
  g_me_w_odd = wo;
  return 0;
}

RAGK_API int ragk_mlp_engine_set_nt(int nt) {
  g_me_nt = nt ? 1 : 0;
  return 0;
}

// stage stamps of every workgroup into a [G][8] u64 buffer (nullptr = off; A/B tooling only)
RAGK_API int ragk_mlp_engine_set_stamps(void* p) {
  g_me_stamps = (unsigned long long*)p;
  return 0;
}

// xn != nullptr: x given. Otherwise the fused post-attention tail: P [S][H] fp32 o_proj slabs, gamma, eps
// (h += bf16(sum P); x = rmsnorm(h) * gamma, add_partials_rmsnorm's math, inside the launch).
// err: device error word; err_host: device address of a host-mapped word (may be null); tmo: device word
// holding the deadline in s_memrealtime ticks (0 = default).
RAGK_API int ragk_mlp_engine(const void* xn, const float* P, int S, const void* gamma, float eps, const void* wgu,
                             const void* wd, void* h, void* act, void* ctr, void* err, void* err_host, const void* tmo,
                             int M, int H, int I, int G, hipStream_t st) {
  if (!ragk_mlp_engine_ok(M, H, I, G)) return (int)hipErrorInvalidValue;
  if (!wgu || !wd || !h || !act || !ctr || !err || !tmo || (!xn && (!P || !gamma || S < 1 || H % 4)))
    return (int)hipErrorInvalidValue;
  MlpArgs a{(const bf16_t*)xn, xn ? nullptr : P, (const bf16_t*)gamma, eps, S, (const bf16_t*)wgu,
            (const bf16_t*)wd, (bf16_t*)h, (bf16_t*)act, (unsigned long long*)ctr, (unsigned*)err,
            (unsigned*)err_host, (const unsigned*)tmo, g_me_stamps, H, I, g_me_w_even, g_me_w_odd};
  if (g_me_nt)
    hipLaunchKernelGGL(mlp_engine_kernel<true>, dim3(G), dim3(ME_THREADS), 0, st, a);
  else
    hipLaunchKernelGGL(mlp_engine_kernel<false>, dim3(G), dim3(ME_THREADS), 0, st, a);
  return (int)hipGetLastError();
}

// bytes of the workspace counters the host allocates zeroed and re-arms after an error (the error word and
// the timeout word follow them: ops/native.py _me_workspace)
RAGK_API int ragk_mlp_engine_ctr_bytes() { return (ME_SHARDS + 1) * ME_CTR_STRIDE * 8; }

// Host-mapped, coherent pinned words (64 B): the kernels' error reports the engine reads after every step
// without a device sync. Returns the host pointer (null on failure); ragk_host_word_dev gives the device one.
RAGK_API void* ragk_host_word_alloc() {
  void* p = nullptr;
  if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
  memset(p, 0, 64);
  return p;
}
RAGK_API void* ragk_host_word_dev(void* host) {
  void* d = nullptr;
  if (!host || hipHostGetDevicePointer(&d, host, 0) != hipSuccess) return nullptr;
  return d;
}
RAGK_API int ragk_host_word_free(void* host) { return host ? (int)hipHostFree(host) : 0; }
