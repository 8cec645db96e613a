// Resident command worker of the device state store (csrc/include/ahv/store.h).
//
// One workgroup of three waves on one CU:
//
//   wave 0 — command wave: polls the command ring (512-byte slots in fine-grained
//            device memory the host writes through the PCIe BAR), executes each
//            command against the HBM tables and writes its result slot.  An
//            audit capture is only *recorded* here (delta row, chain links) and
//            queued for wave 1, so lifecycle / saga / liability commands that
//            follow are answered while the digest is still being computed.
//   wave 1 — hash engine: pops capture jobs from an LDS ring in order, stages the
//            record into LDS as SHA-256 message words with the parent digest
//            spliced in (all 64 lanes), runs the serial compression on lane 0
//            (the chain is inherently serial: ≈2.4 µs per 64-byte block on one
//            lane, scripts/exp/doorbell2.hip) and completes the capture's result.
//
// Commands that read audit state wholesale (FLUSH, FREE_ROWS, NOP = host drain,
// delta reads) wait until wave 1 has drained (`needs_drain`); those that read one
// session's (Merkle root, verify, terminate, header read) wait only for that
// session's queued captures (`session_drain`).
//
// Measured transport (scripts/exp/doorbell2.hip): one host→device→host round
// trip of a 512-byte command ≈3.1 µs p50, vs ≈12 µs for a kernel launch + sync.
//
// Lifetime: a resident workgroup shares its hardware queue with whatever streams
// HIP maps there, so it must not linger — kernels queued behind it (and a device
// synchronize) wait until it exits.  It exits after `idle_ticks` of the 100 MHz
// real-time counter without a command, after `max_ticks` in total, or on
// OP_STOP; the host relaunches it on the next command.  Both waves reach the
// exit: wave 0 drains wave 1, raises `stop`, and waits for wave 1's goodbye
// before clearing the host-visible `alive` word.
//
// Memory: results and bulk outputs go to pinned host memory with system-scope
// stores, the sequence word last after a system release fence; `tail` (pinned
// host memory) carries the next expected sequence number across relaunches.
// Waves hand off through LDS with workgroup-scope release/acquire.
#include <hip/hip_runtime.h>

#include "ahv/store.h"

namespace ahv {
namespace store {

constexpr int kJobs = 64;  // LDS capture-job ring

// Optional timeline (AHV_STORE_TRACE=<entries>): per command [seq+1, op | prefix blocks
// << 32 | waited ticks << 40, t_seen, t_done] at trace[4·(seq mod cap)], per hash-engine
// job [seq+1, blocks | skipped << 8 | batch << 16 | stage << 24 | hash << 44, t_start,
// t_end] at trace[4·(cap + seq mod cap)], per provisional Merkle tree (keyed by the
// capture job after which it ran) [seq+1, leaves | done << 8 | cached << 9, t_start,
// t_end] at trace[4·(2·cap + seq mod cap)], per helper-wave job [seq+1, mode (1 whole record, 2
// prefix) | blocks << 8 | helper << 16, t_start, t_end] at trace[4·(3·cap + seq mod cap)];
// s_memrealtime ticks (100 MHz), pinned memory.
__device__ __forceinline__ void trace_put(uint64_t* tr, int64_t cap, int64_t half, uint64_t seq, uint64_t a,
                                          uint64_t t0, uint64_t t1) {
  if (tr == nullptr || cap <= 0) return;
  uint64_t* e = tr + 4 * (half * cap + static_cast<int64_t>(seq % static_cast<uint64_t>(cap)));
  __hip_atomic_store(e + 1, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(e + 2, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(e + 3, t1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(e, seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
constexpr uint64_t kFreeScan = 8192;  // session / delta rows a FREE_ROWS checks against the queue (longer: full drain)

__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t lds_acquire(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Publication of a result slot: its words are system-scope stores to pinned host
// memory, and the host only needs them to land before the sequence word.  With
// feature bit 32 (`light`, default on; AHV_STORE_LIGHT_PUBLISH=0 turns it off) the command wave's per-command publication is a wait
// for the wave's outstanding stores (vmcnt 0) instead of a system-scope release,
// whose L2 write-back of every dirty table line is paid on each command; table
// rows still reach other agents through the full releases of the wholesale
// commands (FLUSH, the host's drain NOP, FREE_ROWS — needs_drain) and of the
// kernel's exit.  Captures (hash engine, payload bytes) keep the full release.
__device__ __forceinline__ void publish_fence(bool light) {
  if (light) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt(0), expcnt/lgkmcnt unconstrained
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // and no compiler motion of the seq store above it
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
}

// Per-job prefix state (see the header): wave 1 takes a job — CAS 0 → 3, or waits
// for a running prefix (1) to become ready (2).  `ps` is LDS.
__device__ __forceinline__ uint32_t lds_cas(uint32_t* p, uint32_t expect, uint32_t want) {
  __hip_atomic_compare_exchange_strong(p, &expect, want, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
  return expect;  // the value found (== the old expect on success)
}
__device__ __forceinline__ void take_job(uint32_t* ps) {
  if (lds_cas(ps, 0u, 3u) == 1u) {
    while (lds_acquire(ps) != 2u) __builtin_amdgcn_s_sleep(1);
  }
}

// ------------------------------------------------------- batched hash engine
//
// When several captures are queued, the hash engine takes the longest prefix of
// the queue whose jobs belong to distinct sessions (so every job's parent digest
// is already final — the queue is in command order) and hashes it one job per
// lane: up to 64 independent chains advance together instead of one lane doing
// all the rounds while 63 wait.  Each lane stages its own record into a private
// LDS window as big-endian message words (all its loads issued back to back),
// splices the parent's quoted digest in, compresses its blocks and completes its
// capture's result slot.  Windows are kBatchStride = 16·16+1 words apart, so
// when the 64 lanes read word k of their current block they hit 64 different
// banks.  Records longer than kBatchBlocks blocks end the batch (the single-job
// path takes them).
constexpr int kBatchBlocks = 16;
constexpr int kBatchStride = kBatchBlocks * 16 + 1;

__device__ __forceinline__ int64_t job_blocks(const HashJob& j) { return (j.len + 9 + 63) / 64; }

// Number of jobs from jobs[done % kJobs ...] the batch takes (≤ avail, ≤ 64);
// wave-uniform.  `sess` is 64 words of LDS scratch.
__device__ int batch_size(const HashJob* jobs, uint32_t done, uint32_t avail, int32_t* sess, int lane) {
  const bool mine = static_cast<uint32_t>(lane) < avail;
  const HashJob* j = &jobs[(done + lane) % kJobs];
  const int32_t s = mine ? static_cast<int32_t>(j->s) : -1;
  sess[lane] = s;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  bool ok = mine && job_blocks(*j) <= kBatchBlocks;
  for (int k = 0; ok && k < lane; ++k) ok = sess[k] != s;
  const uint64_t bad = __ballot(!ok);
  return bad ? __builtin_ctzll(bad) : 64;
}

// One lane's record of a batch: staged into its window `w` with the parent's quoted
// digest spliced in, then compressed (from the prefix wave's midstate when there is
// one).  `skip`: blocks taken from the midstate.
__device__ __forceinline__ void hash_one(const Tables& t, const HashJob& j, uint32_t* w, uint32_t* kw, uint32_t h[8], int64_t& skip) {
  const uint64_t len = static_cast<uint64_t>(j.len);
  const int64_t nblk = job_blocks(j);
  const int64_t nw = nblk * 16;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(t.payload + j.off);
  // stage: independent system-scope loads of the host-written record, all in flight together
  for (int64_t i = 0; i < nw; ++i) {
    const uint64_t b = 4 * static_cast<uint64_t>(i);
    uint32_t x = 0;
    if (b + 4 <= len) {
      x = bswap32(ld32f(s32 + i));
    } else if (b < len) {
      x = bswap32(ld32f(s32 + i)) & (0xffffffffu << (8 * (4 - static_cast<uint32_t>(len - b))));
    }
    if (b <= len && len < b + 4) x |= 0x80u << (8 * (3 - (len - b)));
    if (i == nw - 2) x |= static_cast<uint32_t>((len * 8) >> 32);
    if (i == nw - 1) x |= static_cast<uint32_t>(len * 8);
    w[i] = x;
  }
  // parent digest: the previous delta of the chain (final: earlier in the queue,
  // hashed by an earlier batch) or the session's chain head for turn 1
  if (j.hole >= 0) {
    const uint32_t* head = j.prev >= 0 ? t.d_hash + 8 * j.prev : t.s_head + 8 * j.s;
    uint32_t hd[8];
    load8(head, hd);
    uint8_t* src = t.payload + j.off;
    uint8_t* lb = reinterpret_cast<uint8_t*>(w);
    auto put = [&](int k, uint32_t ch) {
      const uint64_t b = static_cast<uint64_t>(j.hole) + k;
      src[b] = static_cast<uint8_t>(ch);  // the stored record is completed too
      lb[(b & ~uint64_t(3)) | (3 - (b & 3))] = static_cast<uint8_t>(ch);
    };
    put(0, 0x22u);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
#pragma unroll
      for (int e = 0; e < 8; ++e) put(1 + 8 * q + e, hex_nibble((hd[q] >> (28 - 4 * e)) & 15u));
    }
    put(65, 0x22u);
  }
  skip = j.mid_blocks > 0 && j.mid_blocks < nblk ? j.mid_blocks : 0;
  if (skip) {
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = j.mid[k];
  } else {
    sha256_init(h);
  }
  // per block: message schedule (+K) into the lane's K+W row, then the rounds
  // (the split form keeps the round state in registers; see sha256_rounds_kw)
  for (int64_t b = skip; b < nblk; ++b) {
    sha256_expand_kw(w + 16 * b, kw);
    sha256_rounds_kw(h, kw);
  }
}

// The helper's whole-record digest of a speculated link (HashJob::spec), usable
// when the parent digest its hole held equals the parent's final digest: the
// previous delta's row (earlier in the queue, so already done) or, for the
// chain's first hole, the session head.
__device__ __forceinline__ bool spec_link_ok(const Tables& t, const HashJob& j) {
  if (!j.full) return false;
  if (j.hole < 0) return true;  // a null-parent record (turn 1): its digest depends on its bytes only
  const uint32_t* head = j.prev >= 0 ? t.d_hash + 8 * j.prev : t.s_head + 8 * j.s;
  uint32_t hd[8];
  load8(head, hd);
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 8; ++k) ok = ok && hd[k] == j.ppar[k];
  return ok;
}

// Lane `lane` < n hashes job jobs[(done + lane) % kJobs] and completes it.
__device__ void hash_batch(const Tables& t, const HashJob* jobs, uint32_t done, int n, uint32_t* win,
                           uint32_t* kwrows, uint64_t* res, int64_t nslots, int lane, bool light, uint64_t* tr,
                           int64_t tcap) {
  if (lane >= n) return;
  const uint64_t tj0 = __builtin_amdgcn_s_memrealtime();
  const HashJob& j = jobs[(done + lane) % kJobs];
  uint32_t h[8];
  int64_t nblk = job_blocks(j), skip = 0;
  if (spec_link_ok(t, j)) {  // a helper hashed the whole record and its parent is final and equal
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = j.sdig[k];
    skip = nblk;
  } else {
    hash_one(t, j, win + kBatchStride * lane, kwrows + kKwStride * lane, h, skip);
  }
  store8(t.d_hash + 8 * j.d, h);
  store8(t.s_head + 8 * j.s, h);
  uint64_t* r = res + (j.seq % static_cast<uint64_t>(nslots)) * kResWords;
#pragma unroll
  for (int k = 0; k < 8; ++k) out64(r + 2 + k, h[k]);
  out64(r + 10, 0);
  out64(r + 11, 0);
  out64(r + 12, static_cast<uint64_t>(nblk) | (static_cast<uint64_t>(n) << 32));  // blocks | batch size
  out64(r + 1, ST_OK);
  publish_fence(light);  // digest rows + result words before the sequence word
  out64(r, j.seq + 1);
  trace_put(tr, tcap, 1, j.seq,
            (static_cast<uint64_t>(nblk) & 0xff) | (static_cast<uint64_t>(skip & 0xff) << 8) |
                (static_cast<uint64_t>(n) << 16),
            tj0, __builtin_amdgcn_s_memrealtime());
}

// ------------------------------------------------------- ring lookahead
//
// Feature 256: the helper waves read the command ring past the command wave
// (`cw_next`, published after each command) and hash the captures they find there
// as whole records — a turn-1 record (its digest depends on its bytes only) or a
// link whose predicted parent the host already wrote into the hole — into a small
// LDS table.  The command wave, queuing the capture's job later, takes a ready
// digest with it (the job starts `full`, and the engine only has to check the
// parent, spec_link_ok); a digest that finishes after its job was queued is handed
// to the job if no wave has taken it yet.  Per-call pipelines post their captures
// faster than the command wave works through create / join / activate, so the
// records hash while those commands run instead of after.  Entry states: 0 free,
// 1 hashing, 2 ready, 3 not hashable here, 4 being handed over, 5 hashing for a job
// the command wave queued meanwhile (the job waits, claimed, until the helper completes it).
constexpr int kPre = 8;
constexpr int kAheadSlots = 4;  // slots a scan looks at (16 lanes each: a capture uses ≤ 16 words)

struct PreTab {
  uint32_t st[kPre];
  uint64_t seq[kPre];
  uint32_t dig[kPre][8];
  uint32_t par[kPre][8];
  uint32_t lock;     // one helper scans at a time
  uint64_t cw_next;  // the command wave's next sequence number
};

__device__ __forceinline__ uint64_t lds_acquire64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Leader: give entry e's digest (state 4, held by the caller) to its queued job,
// if the job is still untaken (pstate 0 → 1 → 2); the job is re-identified by its
// sequence number after the claim (its ring slot may have been reused).
__device__ void pre_deliver(PreTab& P, int e, HashJob* jobs, uint32_t* pstate, const uint32_t* q_head,
                            const uint32_t* q_done) {
  const uint64_t seq = P.seq[e];
  const uint32_t d0 = lds_acquire(q_done), h = lds_acquire(q_head);
  for (uint32_t p = d0; p != h; ++p) {
    HashJob* jp = &jobs[p % kJobs];
    if (jp->seq != seq) continue;
    if (lds_cas(&pstate[p % kJobs], 0u, 1u) != 0u) return;  // taken (engine / helper) or done
    if (jp->seq != seq) {  // the slot was reused before the claim: give it back
      lds_release(&pstate[p % kJobs], 0u);
      return;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      jp->sdig[k] = P.dig[e][k];
      jp->ppar[k] = P.par[e][k];
    }
    jp->full = 1;
    lds_release(&pstate[p % kJobs], 2u);
    return;
  }
}

// Leader: entries the command wave has passed — a ready digest goes to its job
// (if still useful), then the entry is freed.
__device__ void pre_sweep(PreTab& P, uint64_t cw, HashJob* jobs, uint32_t* pstate, const uint32_t* q_head,
                          const uint32_t* q_done) {
  for (int e = 0; e < kPre; ++e) {
    const uint32_t sv = lds_acquire(&P.st[e]);
    if ((sv != 2u && sv != 3u) || P.seq[e] >= cw) continue;
    if (lds_cas(&P.st[e], sv, 4u) != sv) continue;
    if (sv == 2u) pre_deliver(P, e, jobs, pstate, q_head, q_done);
    lds_release(&P.st[e], 0u);
  }
}

// One lookahead pass of a helper wave; true when it hashed a record.
__device__ bool lookahead(const Lanes& L, const Tables& t, const uint64_t* ring, int64_t nslots, uint32_t* w,
                          int32_t max_blocks, PreTab& P, HashJob* jobs, uint32_t* pstate, const uint32_t* q_head,
                          const uint32_t* q_done, uint64_t* tr, int64_t tcap, int hw) {
  const int lane = L.lane;
  int locked = 0;
  if (lane == 0) locked = lds_cas(&P.lock, 0u, 1u) == 0u ? 1 : 0;
  locked = __shfl(locked, 0);
  if (!locked) return false;
  const uint64_t cw = lds_acquire64(&P.cw_next);
  if (lane == 0) pre_sweep(P, cw, jobs, pstate, q_head, q_done);
  // lane → word (lane & 15) of slot cw + (lane >> 4); a capture uses ≤ 16 slot words
  const int base = lane & ~15, wi = lane & 15;
  const uint64_t sq = cw + static_cast<uint64_t>(lane >> 4);
  const uint64_t v0 = ld_sys(ring + (sq % static_cast<uint64_t>(nslots)) * kSlotWords + wi);
  const uint64_t w0 = __shfl(v0, base), w1 = __shfl(v0, base + 1), w2 = __shfl(v0, base + 2);
  const uint32_t nwr = static_cast<uint32_t>(w1 >> 32) & 0x7fu;
  const uint64_t v = static_cast<uint32_t>(wi) < nwr ? v0 : 0ull;
  uint64_t x = (wi == 0 || wi == 2) ? 0ull : slot_mix(v, static_cast<uint64_t>(wi));
  for (int o = 8; o > 0; o >>= 1) x ^= __shfl_xor(x, o);
  const uint64_t off = __shfl(v0, base + 7), len = __shfl(v0, base + 8);
  const int64_t hole = static_cast<int64_t>(__shfl(v0, base + 9));
  const uint64_t flags = __shfl(v0, base + 10);
  const uint64_t nblk = (len + 9 + 63) / 64;
  const bool cand = w0 == sq + 1 && static_cast<uint32_t>(w1) == OP_DELTA_CAPTURE && nwr >= 10 && nwr <= 16 &&
                    x == w2 && (hole < 0 || (flags & 1u)) && nblk <= static_cast<uint64_t>(max_blocks) &&
                    off + len <= static_cast<uint64_t>(t.cap.B) && len > 0;
  const uint64_t cb = __ballot(cand && wi == 0);
  int pick_g = -1, pick_e = -1;
  if (lane == 0) {
    for (int g = 0; g < kAheadSlots && pick_g < 0; ++g) {
      if (!((cb >> (16 * g)) & 1ull)) continue;
      const uint64_t sg = cw + static_cast<uint64_t>(g);
      bool have = false;
      for (int e = 0; e < kPre; ++e) have = have || (lds_acquire(&P.st[e]) != 0u && P.seq[e] == sg);
      if (have) continue;
      for (int e = 0; e < kPre; ++e) {
        if (lds_cas(&P.st[e], 0u, 1u) == 0u) {
          P.seq[e] = sg;
          pick_g = g;
          pick_e = e;
          break;
        }
      }
      break;  // no free entry: nothing more this pass
    }
    lds_release(&P.lock, 0u);
  }
  pick_g = __shfl(pick_g, 0);
  pick_e = __shfl(pick_e, 0);
  if (pick_g < 0) return false;
  const uint64_t th0 = __builtin_amdgcn_s_memrealtime();
  HashJob jb;
  jb.off = static_cast<int64_t>(__shfl(off, 16 * pick_g));
  jb.len = static_cast<int64_t>(__shfl(len, 16 * pick_g));
  jb.hole = __shfl(hole, 16 * pick_g);
  jb.spec = jb.hole >= 0 ? 1 : 0;
  uint32_t dig[8] = {0, 0, 0, 0, 0, 0, 0, 0}, par[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  bool whole;
  if (jb.hole >= 0) {
    whole = capture_spec_full(L, t, jb, w, max_blocks, dig, par);
  } else {
    const int64_t nb = (jb.len + 9 + 63) / 64;
    whole = stage_words(L, t.payload + jb.off, static_cast<uint64_t>(jb.len), w, 16 * max_blocks) >= 0;
    if (whole) sha256_lds_blocks_par(L, w, nb, dig);
    L.sync();
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      P.dig[pick_e][k] = dig[k];
      P.par[pick_e][k] = par[k];
    }
    const uint64_t sg = P.seq[pick_e];
    const uint32_t fin = whole ? 2u : 3u;
    if (lds_cas(&P.st[pick_e], 1u, fin) == 5u) {
      // the command wave queued this capture while we hashed and bound the job to us
      // (pstate 1): complete it — with the digest, or without (the engine re-hashes)
      // (the command wave binds before it publishes the job: wait for it to appear;
      // bounded, so a binding that was undone can never hold this wave)
      bool found = false;
      for (int tries = 0; !found && tries < (1 << 16); ++tries) {
        const uint32_t d0 = lds_acquire(q_done), h = lds_acquire(q_head);
        for (uint32_t p = d0; p != h; ++p) {
          HashJob* jp = &jobs[p % kJobs];
          if (jp->seq != sg || lds_acquire(&pstate[p % kJobs]) != 1u) continue;
          if (whole) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              jp->sdig[k] = dig[k];
              jp->ppar[k] = par[k];
            }
            jp->full = 1;
          }
          lds_release(&pstate[p % kJobs], 2u);
          found = true;
          break;
        }
        if (!found) __builtin_amdgcn_s_sleep(1);
      }
      lds_release(&P.st[pick_e], 0u);
    } else {
      // the command wave may have queued this capture meanwhile: hand the digest over
      const uint64_t cw2 = lds_acquire64(&P.cw_next);
      if (sg < cw2 && lds_cas(&P.st[pick_e], fin, 4u) == fin) {
        if (whole) pre_deliver(P, pick_e, jobs, pstate, q_head, q_done);
        lds_release(&P.st[pick_e], 0u);
      }
    }
    trace_put(tr, tcap, 3, sg,
              static_cast<uint64_t>(whole ? 5 : 6) | (static_cast<uint64_t>((jb.len + 9 + 63) / 64 & 0xff) << 8) |
                  (static_cast<uint64_t>(hw) << 16),
              th0, __builtin_amdgcn_s_memrealtime());
  }
  return true;
}

__global__ __launch_bounds__(256) void store_worker_kernel(Tables t, const uint64_t* ring, int64_t nslots,
                                                           uint64_t* res, uint8_t* bulk, uint64_t* alive,
                                                           int64_t* tail, uint64_t idle_ticks, uint64_t max_ticks,
                                                           int speculate, uint64_t* tr, int64_t tcap) {
  __shared__ uint64_t inl[kInlineWords];
  __shared__ uint32_t lds1[kLdsWords];      // wave 1: capture message staging
  __shared__ uint32_t kw1[64 * kKwStride];  // wave 1: per-lane K+W schedule rows
  __shared__ uint32_t lds0[kLdsWords / 4];  // wave 0: staging for its own hashing (capture prefixes)
  __shared__ uint32_t kw0[64 * kKwStride];  // wave 0: K+W schedule rows
  __shared__ HashJob jobs[kJobs];
  __shared__ uint32_t batch_win[64 * kBatchStride];  // wave 1: per-lane record windows (batched hashing)
  __shared__ int32_t batch_sess[64];
  // wave 1: the leaf digests of the chain it last extended (session cc_s, cc_n leaves,
  // the last one delta row cc_d), for the provisional Merkle root
  __shared__ uint32_t chain_cache[64 * 8];
  __shared__ int32_t cc_s, cc_n, cc_d;
  // waves 2, 3 (helpers): per-job helper state, and per helper a staging window
  // (≤ kPrefixBlocks blocks) and K+W rows
  constexpr int kPrefixBlocks = 8;
  constexpr uint32_t kHelperScan = 8;  // pending jobs a helper looks at (from the oldest)
  constexpr uint32_t kSpecQueue = 4;   // whole-record hashing only while ≤ this many are pending
  __shared__ uint32_t pstate[kJobs];
  __shared__ uint32_t lds2[2 * 16 * kPrefixBlocks];
  __shared__ uint32_t kw2[2 * kPrefixBlocks * kKwStride];
  __shared__ uint32_t q_head, q_done, stop, bye, bye2, bye3, spec_s;
  __shared__ PreTab ptab;  // ring lookahead (feature 256)
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) {
    for (int e = 0; e < kPre; ++e) {
      ptab.st[e] = 0;
      ptab.seq[e] = 0;
    }
    ptab.lock = 0;
    ptab.cw_next = static_cast<uint64_t>(__hip_atomic_load(tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    q_head = 0;
    q_done = 0;
    stop = 0;
    bye = 0;
    bye2 = 0;
    bye3 = 0;
    spec_s = 0;  // session + 1 whose provisional Merkle root wave 1 is computing (0: none)
    cc_s = -1;
    cc_n = 0;
    cc_d = -1;
  }
  __syncthreads();  // the only workgroup barrier: every wave passes it once

  if (wave >= 2) {
    // ------------------------------------------------------------ helper waves
    // Two helpers (waves 2, 3 — their own SIMDs) claim pending capture jobs the hash
    // engine has not taken (pstate CAS 0 → 1, done = 2):
    //  * a speculated link (the host prefilled the predicted parent digest, `spec`)
    //    while the queue is short (the per-call regime): the whole record is hashed
    //    now, off the chain — the engine only checks the parent (spec_link_ok);
    //  * otherwise the midstate of the blocks before the parent hole (prefix).
    // Under a long queue (many sessions) the engine batches jobs one per lane and
    // the helpers only do prefixes, so a batch never waits on a whole-record hash.
    const int hw = wave - 2;
    uint32_t* hl = lds2 + hw * 16 * kPrefixBlocks;
    uint32_t* hk = kw2 + hw * kPrefixBlocks * kKwStride;
    const Lanes L{lane, 64, hl, hk};
    for (;;) {
      const uint32_t head = lds_acquire(&q_head);
      const uint32_t dn = lds_acquire(&q_done);
      int32_t pick = -1;
      int32_t mode = 0;  // 1 whole record (spec), 2 prefix
      if (lane == 0 && (speculate & (2 | 128)) && head != dn) {
        const uint32_t pend = head - dn;
        const uint32_t lim = pend < kHelperScan ? head : dn + kHelperScan;
        const bool short_q = pend <= kSpecQueue;
        for (uint32_t p = dn; p != lim; ++p) {
          const HashJob* jp = &jobs[p % kJobs];
          const int32_t m = ((speculate & 128) && short_q && jp->spec && job_blocks(*jp) <= kPrefixBlocks) ? 1
                            : ((speculate & 2) && jp->hole >= 64)                                          ? 2
                                                                                                            : 0;
          if (m && lds_acquire(&pstate[p % kJobs]) == 0u && lds_cas(&pstate[p % kJobs], 0u, 1u) == 0u) {
            pick = static_cast<int32_t>(p % kJobs);
            mode = m;
            break;
          }
        }
      }
      pick = __shfl(pick, 0);
      mode = __shfl(mode, 0);
      if (pick < 0) {
        if (lds_acquire(&stop)) break;
        if ((speculate & 256) &&
            lookahead(L, t, ring, nslots, hl, kPrefixBlocks, ptab, jobs, pstate, &q_head, &q_done, tr, tcap, hw))
          continue;
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      const uint64_t th0 = __builtin_amdgcn_s_memrealtime();
      HashJob* jp = &jobs[pick];
      HashJob jb;
      jb.off = jp->off;
      jb.len = jp->len;
      jb.hole = jp->hole;
      jb.spec = jp->spec;
      bool whole = false;
      if (mode == 1) {
        uint32_t dig[8], par[8];
        whole = capture_spec_full(L, t, jb, hl, kPrefixBlocks, dig, par);
        if (whole && lane == 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            jp->sdig[k] = dig[k];
            jp->ppar[k] = par[k];
          }
          jp->full = 1;
        }
      }
      if (!whole && jb.hole >= 64 && (speculate & 2)) {
        uint32_t mid[8];
        const int32_t pb = capture_prefix(L, t, jb, hl, 16 * kPrefixBlocks, kPrefixBlocks, mid);
        if (lane == 0 && pb > 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) jp->mid[k] = mid[k];
          jp->mid_blocks = pb;
        }
      }
      if (lane == 0) {
        const uint64_t seq = jp->seq;
        const int32_t done_blocks = whole ? static_cast<int32_t>(job_blocks(*jp)) : jp->mid_blocks;
        lds_release(&pstate[pick], 2u);
        trace_put(tr, tcap, 3, seq,
                  static_cast<uint64_t>(whole ? 1 : 2) | (static_cast<uint64_t>(done_blocks & 0xff) << 8) |
                      (static_cast<uint64_t>(hw) << 16),
                  th0, __builtin_amdgcn_s_memrealtime());
      }
    }
    if (lane == 0) lds_release(hw == 0 ? &bye2 : &bye3, 1u);
    return;
  }

  if (wave == 1) {
    // ------------------------------------------------------------ hash engine
    const Lanes L{lane, 64, lds1, kw1};
    uint32_t done = 0;
    uint64_t ebusy = static_cast<uint64_t>(__hip_atomic_load(tail + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    uint64_t ejobs = static_cast<uint64_t>(__hip_atomic_load(tail + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    uint64_t e_start = 0;
    uint32_t e_done0 = 0;
    for (;;) {
      const uint32_t head = lds_acquire(&q_head);
      if (e_start) {  // telemetry: the previous pass's busy ticks and jobs (host-visible)
        ebusy += __builtin_amdgcn_s_memrealtime() - e_start;
        ejobs += done - e_done0;
        e_start = 0;
        if (lane == 0) {
          __hip_atomic_store(tail + 3, static_cast<int64_t>(ebusy), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(tail + 4, static_cast<int64_t>(ejobs), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      if (head == done) {
        if (lds_acquire(&stop)) break;
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      e_start = __builtin_amdgcn_s_memrealtime();
      e_done0 = done;
      if ((speculate & 4) && head - done >= 2) {
        // several captures queued: hash the distinct-session prefix one job per lane
        const int nb = batch_size(jobs, done, head - done, batch_sess, lane);
        if (nb >= 2) {
          if (lane < nb) take_job(&pstate[(done + lane) % kJobs]);
          hash_batch(t, jobs, done, nb, batch_win, kw1, res, nslots, lane, false, tr, tcap);
          if (lane == 0) cc_s = -1;
          done += static_cast<uint32_t>(nb);
          L.sync();
          if (lane == 0) lds_release(&q_done, done);
          continue;
        }
      }
      if (lane == 0) take_job(&pstate[done % kJobs]);
      L.sync();  // the job (with any midstate wave 2 wrote) is read after taking it
      const HashJob& j = jobs[done % kJobs];
      uint64_t* r = res + (j.seq % static_cast<uint64_t>(nslots)) * kResWords;
      uint64_t tele = 0;
      uint32_t hd[8];
      if (spec_link_ok(t, j)) {
        // a helper already hashed this record with the parent digest the engine just
        // computed: take its digest (rows and result words as capture_finish writes them)
        const int64_t nb = job_blocks(j);
        if (lane == 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) hd[k] = j.sdig[k];
          store8(t.d_hash + 8 * j.d, hd);
          store8(t.s_head + 8 * j.s, hd);
#pragma unroll
          for (int k = 0; k < 8; ++k) out64(r + 2 + k, hd[k]);
          out64(r + 10, 0);
          out64(r + 11, 0);
          out64(r + 12, static_cast<uint64_t>(nb));
          out64(r + 1, ST_OK);
          tele = (static_cast<uint64_t>(nb) & 0xff) | ((static_cast<uint64_t>(nb) & 0xff) << 8);
        }
      } else {
        capture_finish(L, t, j, r, &tele, hd);
      }
      if (lane == 0) {
        // extend the cached chain (turn 1 starts one; anything else invalidates it)
        const bool extend = j.prev >= 0 && cc_s == static_cast<int32_t>(j.s) && cc_d == static_cast<int32_t>(j.prev) &&
                            cc_n < 64;
        if (j.prev < 0 || extend) {
          const int32_t k = j.prev < 0 ? 0 : cc_n;
#pragma unroll
          for (int q = 0; q < 8; ++q) chain_cache[8 * k + q] = hd[q];
          cc_s = static_cast<int32_t>(j.s);
          cc_n = k + 1;
          cc_d = static_cast<int32_t>(j.d);
        } else {
          cc_s = -1;
        }
        publish_fence(false);  // digest row + result words before the sequence word
        out64(r, j.seq + 1);
        trace_put(tr, tcap, 1, j.seq, tele | (1ull << 16), e_start, __builtin_amdgcn_s_memrealtime());
      }
      ++done;
      // Idle next?  Then compute the chain's provisional Merkle root now, so a
      // terminate / compute_merkle_root that follows finds it ready.  `spec_s`
      // is raised before q_done: a drained command wave sees it and, for the
      // same session, waits for the (abortable, few-µs) tree instead of
      // recomputing it; every other command runs alongside.
      const bool idle = (speculate & 1) && __shfl(static_cast<int>(lds_acquire(&q_head) == done), 0) != 0;  // wave-uniform
      if (lane == 0) {
        if (idle) lds_release(&spec_s, static_cast<uint32_t>(j.s) + 1u);
        lds_release(&q_done, done);
      }
      if (idle) {
        L.sync();  // the leader's cache update is visible to every lane
        const bool hit = cc_s == static_cast<int32_t>(j.s) && cc_d == static_cast<int32_t>(j.d);
        const int64_t n = hit ? static_cast<int64_t>(cc_n) : static_cast<int64_t>(t.d_turn[j.d]);
        const uint64_t tt0 = __builtin_amdgcn_s_memrealtime();
        const bool ok = merkle_provisional(L, t, j.s, j.d, n, lds1, [&] { return lds_acquire(&q_head) != done; },
                                           hit ? chain_cache : nullptr);
        if (lane == 0) lds_release(&spec_s, 0u);  // the s_proot rows precede this release
        if (lane == 0)
          trace_put(tr, tcap, 2, j.seq,
                    static_cast<uint64_t>(n & 0xff) | (ok ? 256ull : 0ull) | (hit ? 512ull : 0ull), tt0,
                    __builtin_amdgcn_s_memrealtime());
      }
    }
    if (lane == 0) lds_release(&bye, 1u);
    return;
  }

  // ------------------------------------------------------------ command wave
  const Lanes L{lane, 64, lds0, kw0, &spec_s};
  uint64_t next = static_cast<uint64_t>(__hip_atomic_load(tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  uint32_t queued = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t last = t0;
  // telemetry accumulates across relaunches (tail[1..4] persist in pinned memory)
  uint64_t busy = static_cast<uint64_t>(__hip_atomic_load(tail + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  uint64_t ncmd = static_cast<uint64_t>(__hip_atomic_load(tail + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  // feature bit 64 (default on; AHV_STORE_SLOT_PREFETCH=0 off): the next slot is loaded while the current command executes, so
  // a worker running behind the host does not pay a fine-grained read round trip
  // between commands (a stale or torn prefetch is simply re-polled)
  uint64_t pre = 0;
  bool have_pre = false;
  for (;;) {
    const uint64_t* slot = ring + (next % static_cast<uint64_t>(nslots)) * kSlotWords;
    uint64_t w;
    if (have_pre) {
      w = pre;
      have_pre = false;
    } else {
      w = ld_sys(slot + lane);
    }
    const uint64_t seq = __shfl(w, 0);
    if (seq != next + 1) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (now - last > idle_ticks || now - t0 > max_ticks) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    // the host writes only the words in use (count in w[1]'s high half); the rest of
    // the slot still holds an older command and reads as zero
    const uint32_t nwr = static_cast<uint32_t>(__shfl(w, 1) >> 32) & 0x7fu;
    const uint64_t v = static_cast<uint32_t>(lane) < (nwr ? nwr : 64u) ? w : 0ull;
    uint64_t x = (lane == 0 || lane == 2) ? 0ull : slot_mix(v, static_cast<uint64_t>(lane));
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o);
    if (x != __shfl(v, 2)) continue;  // torn read of a slot still being written: poll again
    const uint64_t c_start = __builtin_amdgcn_s_memrealtime();
    Cmd c;
    c.op = static_cast<uint32_t>(__shfl(v, 1));
#pragma unroll
    for (int k = 0; k < kArgs; ++k) c.a[k] = __shfl(v, 3 + k);
    if (lane >= 16) inl[lane - 16] = v;
    L.sync();
    c.inl = inl;
    // (feature 512: issued after the command's publication instead — the publication
    // waits for every outstanding vector memory op, a prefetch issued before it too)
    if ((speculate & 64) && !(speculate & 512)) {
      pre = ld_sys(ring + ((next + 1) % static_cast<uint64_t>(nslots)) * kSlotWords + lane);
      have_pre = true;
    }
    // OP_FREE_ROWS of saga / step / vouch-edge / liability rows: the hash engine
    // never touches those tables, so nothing to wait for.  Of session rows: only
    // the queued captures (and a provisional tree) of the sessions being freed —
    // not the engine's whole backlog, which stalled every command behind it for
    // milliseconds once per few hundred released sessions.  Long lists and delta
    // rows (their digests are what the engine writes) still drain it fully.
    const bool free_rows = c.op == OP_FREE_ROWS;
    const bool free_light = (speculate & 16) && free_rows && ((c.a[0] != RK_S && c.a[0] != RK_D) || c.a[1] <= kFreeScan);
    if (free_light && (c.a[0] == RK_S || c.a[0] == RK_D)) {
      // lanes stride over the freed rows (independent loads); each row is compared
      // with the pending jobs' sessions (S) or delta rows (D: a queued job reads its
      // record from the arena and writes its digest row), snapshotted into this
      // wave's scratch.  A provisional tree in flight blocks freeing its session, and
      // any delta rows (it reads its chain's digests).
      const bool drows = c.a[0] == RK_D;
      const IndexList idx = index_list(t, c, c.a[1], c.a[2]);
      const int64_t n = static_cast<int64_t>(c.a[1]);
      int32_t* pend = reinterpret_cast<int32_t*>(lds0);
      for (;;) {
        const uint32_t d0 = __shfl(lds_acquire(&q_done), 0);
        const uint32_t np = queued - d0;  // ≤ kJobs
        // spec_s is raised before q_done is released: read after q_done, it shows any
        // tree started on a job this snapshot already counts as done
        const int32_t sp = static_cast<int32_t>(__shfl(lds_acquire(&spec_s), 0)) - 1;
        if (static_cast<uint32_t>(lane) < np) {
          const HashJob& jb = jobs[(d0 + lane) % kJobs];
          pend[lane] = static_cast<int32_t>(drows ? jb.d : jb.s);
        }
        L.sync();
        bool hit = drows && sp >= 0;
        for (int64_t i = lane; i < n && !hit; i += 64) {
          const int32_t x = idx[i];
          hit = x == sp;
          for (uint32_t k = 0; k < np && !hit; ++k) hit = pend[k] == x;
        }
        L.sync();  // every lane has read `pend` before the next snapshot
        if (__ballot(hit) == 0) break;
        __builtin_amdgcn_s_sleep(1);
      }
    } else if (!free_light && needs_drain(c.op)) {
      while (lds_acquire(&q_done) != queued) __builtin_amdgcn_s_sleep(1);
      if (c.op == OP_FREE_ROWS) {  // no provisional tree still writing a row about to be freed
        while (lds_acquire(&spec_s) != 0u) __builtin_amdgcn_s_sleep(1);
      }
    } else if (session_drain(c.op)) {
      // only this session's captures: lane k checks queued job done+k (≤ kJobs pending)
      const int64_t s = static_cast<int64_t>(c.a[0]);
      for (;;) {
        const uint32_t d0 = lds_acquire(&q_done);
        const bool mine = static_cast<uint32_t>(lane) < queued - d0 && jobs[(d0 + lane) % kJobs].s == s;
        if (__ballot(mine) == 0) break;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    // (a close / Merkle command waits for the tree in flight inside its execution,
    // right before it reads the provisional root: Lanes::wait_tree)
    if (c.op == OP_DELTA_CAPTURE) {
      while (queued - lds_acquire(&q_done) >= static_cast<uint32_t>(kJobs)) __builtin_amdgcn_s_sleep(1);
    }
    if (c.op == OP_ACQUIRE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const uint64_t c_waited = __builtin_amdgcn_s_memrealtime() - c_start;
    uint64_t* r = res + (next % static_cast<uint64_t>(nslots)) * kResWords;
    HashJob job;
    job.mid_blocks = 0;
    const int rc = store_exec(L, t, c, next, r, bulk, &job);
    if (c.op == OP_FLUSH) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    L.sync();
    if (rc == EXEC_DEFERRED) {
      if (lane == 0) {
        uint32_t ps0 = 0u;
        if (speculate & 256) {  // a helper hashed (or is hashing) this record from the ring
          for (int e = 0; e < kPre; ++e) {
            if (ptab.seq[e] != next) continue;
            if (lds_cas(&ptab.st[e], 2u, 4u) == 2u) {
              if (ptab.seq[e] == next) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                  job.sdig[k] = ptab.dig[e][k];
                  job.ppar[k] = ptab.par[e][k];
                }
                job.full = 1;
                ps0 = 2u;  // done: no helper claims it, the engine takes it at once
              }
              lds_release(&ptab.st[e], 0u);
              break;
            }
            if (lds_cas(&ptab.st[e], 1u, 5u) == 1u) {
              // still hashing: the job is queued as claimed (pstate 1), so neither the
              // engine nor the other helper hashes it again — the engine waits for the
              // helper, which completes the job (pstate 2) when its digest is ready
              if (ptab.seq[e] == next) {
                ps0 = 1u;
              } else {  // (the entry moved on meanwhile: undo)
                lds_release(&ptab.st[e], 1u);
              }
              break;
            }
          }
        }
        jobs[queued % kJobs] = job;  // (mid_blocks 0: wave 2 may add a midstate)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        pstate[queued % kJobs] = ps0;
        lds_release(&q_head, queued + 1);  // the capture's global row writes precede this release
      }
      ++queued;
    } else if (lane == 0) {
      // (captures complete payload bytes the host may read by DMA: full release)
      publish_fence((speculate & 32) != 0 && !needs_drain(c.op) && c.op != OP_DELTA_CAPTURE);
      out64(r, next + 1);
    }
    if ((speculate & 64) && (speculate & 512)) {
      pre = ld_sys(ring + ((next + 1) % static_cast<uint64_t>(nslots)) * kSlotWords + lane);
      have_pre = true;
    }
    if (lane == 0) __hip_atomic_store(tail, static_cast<int64_t>(next + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 0) __hip_atomic_store(&ptab.cw_next, next + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    last = __builtin_amdgcn_s_memrealtime();
    if (lane == 0)
      trace_put(tr, tcap, 0, next,
                c.op | (static_cast<uint64_t>(job.mid_blocks & 0xff) << 32) | ((c_waited & 0xffffff) << 40), c_start,
                last);
    ++next;
    // utilisation telemetry (host-visible, pinned): busy ticks of the command wave
    // (decode → result written; waits for the hash engine included) and commands
    busy += last - c_start;
    ++ncmd;
    if (lane == 0) {
      __hip_atomic_store(tail + 1, static_cast<int64_t>(busy), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(tail + 2, static_cast<int64_t>(ncmd), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (rc == EXEC_STOP) break;
  }
  // drain the hash engine, stop it, wait for its goodbye, then release the queue
  while (lds_acquire(&q_done) != queued) __builtin_amdgcn_s_sleep(1);
  if (lane == 0) lds_release(&stop, 1u);
  while (!lds_acquire(&bye) || !lds_acquire(&bye2) || !lds_acquire(&bye3)) __builtin_amdgcn_s_sleep(1);
  if (lane == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(alive, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace store
}  // namespace ahv

// Host-callable launcher (one workgroup: command wave, hash-engine wave, two helper waves).
extern "C" int ahv_store_launch_worker(const ahv::store::Tables* t, const uint64_t* ring, int64_t nslots,
                                       uint64_t* res, uint8_t* bulk, uint64_t* alive, int64_t* tail,
                                       uint64_t idle_ticks, uint64_t max_ticks, int speculate,
                                       uint64_t* trace, int64_t trace_cap, hipStream_t stream) {
  hipLaunchKernelGGL(ahv::store::store_worker_kernel, dim3(1), dim3(256), 0, stream, *t, ring, nslots, res, bulk,
                     alive, tail, idle_ticks, max_ticks, speculate, trace, trace_cap);
  return static_cast<int>(hipGetLastError());
}
