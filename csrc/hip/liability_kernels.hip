// Batched joint-liability kernels (SURVEY §2.14 K03–K07).
//
// Representation: a session's participants have local indices 0..15 (the
// reference's max_participants default is 10; rows are padded to 16), its vouch
// edges live in creation order in a CSR edge list, and for scoring the live
// bonds are summed into a dense 16×16 fp64 tile (row = voucher, col = vouchee).
//
// K03/K04 on MFMA: with a wave per session tile, the column sums (Σ bonded for
// each vouchee → σ_eff) and row sums (exposure of each voucher) are two chains of
// four v_mfma_f64_16x16x4_f64 against an all-ones operand.  fp64 MFMA sums the
// 16 terms in tile order; the reference sums in vouch-creation order, so the MFMA
// path agrees to within an ulp-level tolerance while `sigma_eff_csr` (one lane
// per vouchee, creation order) is the bit-exact path.
#include <cstdlib>
#include <string>

#include "ahv/kernels.h"
#include "ahv/launch.h"
#include "ahv/semantics.h"

namespace ahv {

typedef double f64x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int kBlock = 256;
inline dim3 grid1(int64_t n, int per_block = kBlock) {
  const int64_t b = (n + per_block - 1) / per_block;
  return dim3(static_cast<uint32_t>(b > 0 ? b : 1));
}
// Both words are loaded unconditionally: a short-circuit `active[e] && expiry[e]…`
// makes the expiry load wait for the active byte (two dependent round trips).
AHV_HD bool live_edge(const uint8_t* active, const int64_t* expiry, int64_t e, int64_t now) {
  const uint8_t act = active[e];
  const int64_t x = expiry != nullptr ? expiry[e] : -1;
  return act != 0 && (x < 0 || now <= x);
}
// σ of the batched encoding: NaN marks an agent absent from agent_scores, which the
// reference reads as 0.0 (as the slash kernel does), so no caller has to scrub NaNs.
AHV_HD double score_or_zero(double x) { return x != x ? 0.0 : x; }
}  // namespace

// ------------------------------------------------------------ K03/K04 MFMA

__global__ __launch_bounds__(64) void bond_tiles_mfma_kernel(BondTileArgs a) {
  const int64_t s = blockIdx.x;
  if (s >= a.sessions) return;
  const int l = threadIdx.x;
  const int r = l >> 4, c = l & 15;
  const double* T = a.tiles + s * kTile * kTile;
  f64x4 col = {0.0, 0.0, 0.0, 0.0};
  f64x4 row = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    // B operand (k = voucher 4t+r, j = vouchee c): Σ_k 1·T[k][j] → column sums
    const double b = T[(4 * t + r) * kTile + c];
    col = __builtin_amdgcn_mfma_f64_16x16x4f64(1.0, b, col, 0, 0, 0);
    // A operand (i = voucher c, k = vouchee 4t+r): Σ_k T[i][k]·1 → row sums
    const double av = T[c * kTile + 4 * t + r];
    row = __builtin_amdgcn_mfma_f64_16x16x4f64(av, 1.0, row, 0, 0, 0);
  }
  // D layout: col = lane&15, row = (lane>>4) + 4*reg.  Every row of `col` holds the
  // column sums; lanes 0..15 (reg 0) write them.  Column 0 of `row` holds every
  // row sum: lanes 0,16,32,48 write rows r + 4*reg.
  if (r == 0) {
    const double bonded = col[0];
    a.bonded_in[s * kTile + c] = bonded;
    a.sigma_eff[s * kTile + c] = sigma_eff_combine(a.sigma[s * kTile + c], a.omega[s], bonded);
  }
  if (c == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a.exposure[s * kTile + r + 4 * q] = row[q];
      // fused agent-indexed scatter (X01 input): one hardware fp64 atomic per
      // participant instead of a separate index_add pass over [S, 16]
      if (a.members) unsafeAtomicAdd(a.agent_exposure + a.members[s * kTile + r + 4 * q], row[q]);
    }
  }
}

void launch_bond_tiles(const BondTileArgs& a, hipStream_t st) {
  if (a.sessions <= 0) return;
  hipLaunchKernelGGL(bond_tiles_mfma_kernel, dim3(static_cast<uint32_t>(a.sessions)), dim3(64), 0, st, a);
  check_hip(hipGetLastError(), "bond_tiles_mfma_kernel");
}

void bond_tiles_host(const BondTileArgs& a) {
  for (int64_t s = 0; s < a.sessions; ++s) {
    const double* T = a.tiles + s * kTile * kTile;
    for (int j = 0; j < kTile; ++j) {
      double cs = 0.0, rs = 0.0;
      for (int k = 0; k < kTile; ++k) {
        cs += T[k * kTile + j];
        rs += T[j * kTile + k];
      }
      a.bonded_in[s * kTile + j] = cs;
      a.sigma_eff[s * kTile + j] = sigma_eff_combine(a.sigma[s * kTile + j], a.omega[s], cs);
      a.exposure[s * kTile + j] = rs;
      if (a.members) a.agent_exposure[a.members[s * kTile + j]] += rs;
    }
  }
}

// ------------------------------------------------- K03/K04 fused (CSR → MFMA)
// Operand layouts of v_mfma_f64_16x16x4_f64 (as in bond_tiles_mfma_kernel):
// lane l = 16·r + c supplies A[i=c][k=r] and B[k=r][j=c]; it receives
// D[row=r+4q][col=c] in register q.  A wave owns 16 consecutive sessions (their
// edges are one contiguous CSR range) and walks it 64 edges at a time.
//
// Load: lane 16·r + c reads edge base + 4c + r — the 64 lanes cover 64
// consecutive edges, so the loads stay fully coalesced — packing liveness,
// voucher and vouchee into one word.  Chunk u (edges base+4u … base+4u+3) needs,
// in every lane of row r, edge 4u + r, which lane 16·r + u holds: one DPP
// row_newbcast:u per 32-bit value hands it to the whole row (VALU, no LDS).
// Then A is the edge's bond if it lies in session c's CSR range [off_c, off_c+1)
// — each lane tests its own session, no search — and B is whether its vouchee
// (voucher) is c.  Two MFMAs per chunk accumulate Σbonded per (session, vouchee)
// and per (session, voucher).  The next 64 edges are loaded before the current
// ones are consumed.  In-chunk sums are MFMA-ordered, so results agree with the
// creation-order reference to ulp level (the CSR kernel stays the bit-exact path).

constexpr int kFusedWaves = 4;      // waves per block
constexpr int kFusedSessions = 16;  // sessions per wave (A rows)

struct FusedLane {
  int32_t base;   // first edge of the batch
  int32_t off_c, off_c1;
  uint32_t c, r;
};

__device__ __forceinline__ void fused_load(const BondFusedArgs& a, int32_t g, int32_t e1, uint32_t& meta, double& bond) {
  meta = 0u;
  bond = 0.0;
  if (g < e1) {
    const uint32_t vr = a.voucher[g], ve = a.vouchee[g];  // one round trip with the liveness words
    const bool live = live_edge(a.active, a.expiry_us, g, a.now_us);
    meta = live ? (0x10000u | (vr << 8) | ve) : 0u;
    bond = a.bonded[g];
  }
}

template <int U>
__device__ __forceinline__ void fused_chunk(const FusedLane& L, uint32_t meta, uint32_t b_lo, uint32_t b_hi,
                                            f64x4& acc_in, f64x4& acc_out) {
  constexpr int kBcast = 0x150 + U;  // row_newbcast:U
  const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(meta), kBcast, 0xF, 0xF, false));
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(b_lo), kBcast, 0xF, 0xF, false));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(b_hi), kBcast, 0xF, 0xF, false));
  const double b = __hiloint2double(static_cast<int>(hi), static_cast<int>(lo));
  const int32_t g = L.base + 4 * U + static_cast<int32_t>(L.r);
  const double av = ((m >> 16) && g >= L.off_c && g < L.off_c1) ? b : 0.0;
  const double bi = (m & 0xffu) == L.c ? 1.0 : 0.0;
  const double bo = ((m >> 8) & 0xffu) == L.c ? 1.0 : 0.0;
  acc_in = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bi, acc_in, 0, 0, 0);
  acc_out = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bo, acc_out, 0, 0, 0);
}

template <int U0>
__device__ __forceinline__ void fused_quad(const FusedLane& L, uint32_t meta, uint32_t lo, uint32_t hi, f64x4& ai,
                                           f64x4& ao) {
  fused_chunk<U0>(L, meta, lo, hi, ai, ao);
  fused_chunk<U0 + 1>(L, meta, lo, hi, ai, ao);
  fused_chunk<U0 + 2>(L, meta, lo, hi, ai, ao);
  fused_chunk<U0 + 3>(L, meta, lo, hi, ai, ao);
}

__global__ __launch_bounds__(64 * kFusedWaves) void bond_fused_mfma_kernel(BondFusedArgs a) {
  const int wave = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  const int64_t s0 = (static_cast<int64_t>(blockIdx.x) * kFusedWaves + wave) * kFusedSessions;
  if (s0 >= a.sessions) return;  // wave-uniform
  const int64_t s_end = s0 + kFusedSessions < a.sessions ? s0 + kFusedSessions : a.sessions;
  const int32_t e0 = a.offsets[s0], e1 = a.offsets[s_end];
  FusedLane L;
  L.r = static_cast<uint32_t>(l >> 4);
  L.c = static_cast<uint32_t>(l & 15);
  const int64_t sc = s0 + L.c;
  L.off_c = sc < s_end ? a.offsets[sc] : e1;
  L.off_c1 = sc < s_end ? a.offsets[sc + 1] : e1;
  const int32_t my = static_cast<int32_t>(4 * L.c + L.r);  // this lane's edge within a batch
  f64x4 acc_in = {0.0, 0.0, 0.0, 0.0};
  f64x4 acc_out = {0.0, 0.0, 0.0, 0.0};
  uint32_t meta;
  double bond;
  fused_load(a, e0 + my, e1, meta, bond);
  for (int32_t base = e0; base < e1; base += 64) {
    uint32_t meta_n;
    double bond_n;
    fused_load(a, base + 64 + my, e1, meta_n, bond_n);  // next batch in flight
    L.base = base;
    const uint32_t lo = static_cast<uint32_t>(__double2loint(bond));
    const uint32_t hi = static_cast<uint32_t>(__double2hiint(bond));
    const int32_t rem = e1 - base;  // wave-uniform; lanes past e1 carry zeros
    fused_quad<0>(L, meta, lo, hi, acc_in, acc_out);
    if (rem > 16) fused_quad<4>(L, meta, lo, hi, acc_in, acc_out);
    if (rem > 32) fused_quad<8>(L, meta, lo, hi, acc_in, acc_out);
    if (rem > 48) fused_quad<12>(L, meta, lo, hi, acc_in, acc_out);
    meta = meta_n;
    bond = bond_n;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t s = s0 + L.r + 4 * q;
    if (s >= s_end) continue;
    const int64_t o = s * kTile + L.c;  // 64 consecutive doubles per q across the wave
    const double bonded = acc_in[q];
    if (a.bonded_in) a.bonded_in[o] = bonded;
    a.sigma_eff[o] = sigma_eff_combine(score_or_zero(a.sigma[o]), a.omega[s], bonded);
    a.exposure[o] = acc_out[q];
    // X01 input: only members that vouch for someone carry exposure (≈ 60 % of a
    // 16-member row with 8 edges is zero) — adding +0.0 to a non-negative sum is a
    // no-op, so those fp64 atomics are skipped
    if (a.members && acc_out[q] != 0.0) unsafeAtomicAdd(a.agent_exposure + a.members[o], acc_out[q]);
  }
}

void launch_bond_fused(const BondFusedArgs& a, hipStream_t st) {
  if (a.sessions <= 0) return;
  const int64_t per_block = static_cast<int64_t>(kFusedWaves) * kFusedSessions;
  hipLaunchKernelGGL(bond_fused_mfma_kernel, grid1(a.sessions, static_cast<int>(per_block)), dim3(64 * kFusedWaves),
                     0, st, a);
  check_hip(hipGetLastError(), "bond_fused_mfma_kernel");
}

// Host twin: creation-order sums per (session, vouchee) and (session, voucher).
void bond_fused_host(const BondFusedArgs& a) {
  for (int64_t s = 0; s < a.sessions; ++s) {
    double in[kTile] = {0.0}, out[kTile] = {0.0};
    for (int32_t k = a.offsets[s]; k < a.offsets[s + 1]; ++k) {
      if (!live_edge(a.active, a.expiry_us, k, a.now_us)) continue;
      in[a.vouchee[k]] += a.bonded[k];
      out[a.voucher[k]] += a.bonded[k];
    }
    for (int j = 0; j < kTile; ++j) {
      const int64_t o = s * kTile + j;
      if (a.bonded_in) a.bonded_in[o] = in[j];
      a.sigma_eff[o] = sigma_eff_combine(score_or_zero(a.sigma[o]), a.omega[s], in[j]);
      a.exposure[o] = out[j];
      if (a.members) a.agent_exposure[a.members[o]] += out[j];
    }
  }
}

// ------------------------------------------------------ tile build (CSR → dense)
// One wave per session; lane j owns tile entries j, j+64, j+128, j+192 and sums
// the matching live edges in creation order (deterministic).

AHV_HD void build_tile_entry(const VouchCsrArgs& a, int64_t s, int idx) {
  const int v = idx / kTile, e = idx % kTile;
  double acc = 0.0;
  for (int32_t k = a.offsets[s]; k < a.offsets[s + 1]; ++k)
    if (a.voucher[k] == v && a.vouchee[k] == e && live_edge(a.active, a.expiry_us, k, a.now_us)) acc += a.bonded[k];
  a.tiles[s * kTile * kTile + idx] = acc;
}

// Device: the session's edges are staged once in LDS as a (voucher·16 + vouchee)
// key (0xffff = not live: every byte value is a real entry) and the bond; every lane then walks them in
// creation order for its 4 entries — all 64 lanes read the same edge (an LDS
// broadcast) instead of 5 global loads per edge per entry.
constexpr int kTileLdsEdges = 512;

__global__ __launch_bounds__(64) void build_tiles_kernel(VouchCsrArgs a) {
  __shared__ uint16_t s_key[kTileLdsEdges];
  __shared__ double s_bd[kTileLdsEdges];
  const int64_t s = blockIdx.x;
  if (s >= a.sessions) return;
  const int32_t b = a.offsets[s], n = a.offsets[s + 1] - b;
  if (n > kTileLdsEdges) {  // uniform per block
#pragma unroll
    for (int q = 0; q < 4; ++q) build_tile_entry(a, s, threadIdx.x + 64 * q);
    return;
  }
  for (int32_t k = threadIdx.x; k < n; k += 64) {
    const bool live = live_edge(a.active, a.expiry_us, b + k, a.now_us);
    s_key[k] = live ? static_cast<uint16_t>(a.voucher[b + k] * kTile + a.vouchee[b + k]) : 0xffffu;
    s_bd[k] = a.bonded[b + k];
  }
  __syncthreads();
  const uint32_t i0 = threadIdx.x;
  double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
  for (int32_t k = 0; k < n; ++k) {
    const uint32_t key = s_key[k];
    const double bd = s_bd[k];
    if (key == i0) acc0 += bd;
    if (key == i0 + 64) acc1 += bd;
    if (key == i0 + 128) acc2 += bd;
    if (key == i0 + 192) acc3 += bd;
  }
  double* t = a.tiles + s * kTile * kTile;
  t[i0] = acc0;
  t[i0 + 64] = acc1;
  t[i0 + 128] = acc2;
  t[i0 + 192] = acc3;
}
void launch_build_tiles(const VouchCsrArgs& a, hipStream_t st) {
  if (a.sessions <= 0) return;
  hipLaunchKernelGGL(build_tiles_kernel, dim3(static_cast<uint32_t>(a.sessions)), dim3(64), 0, st, a);
  check_hip(hipGetLastError(), "build_tiles_kernel");
}
void build_tiles_host(const VouchCsrArgs& a) {
  for (int64_t s = 0; s < a.sessions; ++s)
    for (int idx = 0; idx < kTile * kTile; ++idx) build_tile_entry(a, s, idx);
}

// --------------------------------------------------- K03 exact (creation order)

AHV_HD void sigma_eff_csr_elem(const VouchCsrArgs& a, int64_t i) {
  const int64_t s = i / kTile;
  const int e = static_cast<int>(i % kTile);
  double contrib = 0.0;
  for (int32_t k = a.offsets[s]; k < a.offsets[s + 1]; ++k)
    if (a.vouchee[k] == e && live_edge(a.active, a.expiry_us, k, a.now_us)) contrib += a.bonded[k];
  a.sigma_eff[i] = sigma_eff_combine(score_or_zero(a.sigma[i]), a.omega[s], contrib);
}
// Device: a 256-thread block owns 16 sessions; thread (session, vouchee) walks
// its session's edges in creation order and adds the live bonds of its vouchee —
// the element form above, the same additions in the same order.  The block's
// edge range is staged in LDS with coalesced loads (liveness precomputed); the
// 16 threads of a session read the same edge (a broadcast), and one pad slot
// per 16 edges puts the 4 sessions of a wave on different banks.  σ and σ_eff
// rows are read/written coalesced, one (session, vouchee) per thread.
constexpr int kSigmaSessions = 16;  // sessions per block (× kTile threads)
constexpr int kSigmaLdsEdges = 2048;

__device__ __forceinline__ int32_t pad_edge(int32_t i) { return i + (i >> 4); }

__global__ __launch_bounds__(kSigmaSessions * kTile) void sigma_eff_csr_kernel(VouchCsrArgs a) {
  __shared__ uint8_t s_ve[kSigmaLdsEdges + kSigmaLdsEdges / 16];
  __shared__ double s_bd[kSigmaLdsEdges + kSigmaLdsEdges / 16];  // 0.0 for a dead edge
  const int64_t s0 = static_cast<int64_t>(blockIdx.x) * kSigmaSessions;
  const int64_t s1 = s0 + kSigmaSessions < a.sessions ? s0 + kSigmaSessions : a.sessions;
  const int64_t i = s0 * kTile + threadIdx.x;  // (session, vouchee) element
  // Everything this thread reads that does not depend on the block's edge range
  // is requested up front, so the σ / ω / own-range loads overlap the range
  // lookup and the edge staging (two dependent memory round trips, not three).
  const bool mine = i < s1 * kTile;
  const int64_t si = mine ? i / kTile : s0;
  double sig = 0.0, om = 0.0;
  int32_t kb = 0, ke = 0;
  if (mine) {
    sig = a.sigma[i];
    om = a.omega[si];
    kb = a.offsets[si];
    ke = a.offsets[si + 1];
  }
  const int32_t e0 = a.offsets[s0], e1 = a.offsets[s1];
  if (e1 - e0 > kSigmaLdsEdges) {  // uniform per block: element form from global memory
    if (mine) sigma_eff_csr_elem(a, i);
    return;
  }
  for (int32_t k = e0 + threadIdx.x; k < e1; k += kSigmaSessions * kTile) {
    const int32_t j = pad_edge(k - e0);
    const uint8_t ve = a.vouchee[k];
    const bool live = live_edge(a.active, a.expiry_us, k, a.now_us);
    s_ve[j] = live ? ve : 0xff;  // a dead edge matches no vouchee
    s_bd[j] = a.bonded[k];
  }
  __syncthreads();
  if (mine) {
    const uint32_t e = static_cast<uint32_t>(i % kTile);
    double contrib = 0.0;
    for (int32_t k = kb - e0; k < ke - e0; ++k) {
      const int32_t j = pad_edge(k);
      if (s_ve[j] == e) contrib += s_bd[j];
    }
    a.sigma_eff[i] = sigma_eff_combine(score_or_zero(sig), om, contrib);
  }
}
void launch_sigma_eff_csr(const VouchCsrArgs& a, hipStream_t st) {
  if (a.sessions <= 0) return;
  hipLaunchKernelGGL(sigma_eff_csr_kernel, grid1(a.sessions, kSigmaSessions), dim3(kSigmaSessions * kTile), 0, st, a);
  check_hip(hipGetLastError(), "sigma_eff_csr_kernel");
}
void sigma_eff_csr_host(const VouchCsrArgs& a) {
  for (int64_t i = 0; i < a.sessions * kTile; ++i) sigma_eff_csr_elem(a, i);
}


// Streaming form (the default K03 exact path): a 16-lane group per session (lane
// j = vouchee j), a wave = 4 consecutive sessions, kStreamSlices such slices per
// wave, and every load of every slice — edge range, σ, ω, then the first 16
// edges, one per lane — issued before the first sum, so a wave keeps ~4 KB in
// flight instead of one dependent round trip at a time (the LDS-staged form
// above spends half its waves' time on the offsets round trip).  The sum needs
// no LDS: DPP row_newbcast:u hands edge u of each 16-lane row (= the group) to
// every lane of the row, so each lane walks its session's edges in creation
// order and adds the live bonds of its own vouchee — the additions, in the
// order, of sigma_eff_csr_elem.  Sessions with more than 16 edges walk further
// chunks in-line (loads on demand).
constexpr int kStreamWaves = 4;

__device__ __forceinline__ uint32_t row_bcast(uint32_t x, int u) {
  // dpp_ctrl row_newbcast:u = 0x150 + u (must be an immediate: unrolled callers)
  switch (u) {
#define AHV_RB(U) case U: return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x150 + U, 0xF, 0xF, false));
    AHV_RB(0) AHV_RB(1) AHV_RB(2) AHV_RB(3) AHV_RB(4) AHV_RB(5) AHV_RB(6) AHV_RB(7)
    AHV_RB(8) AHV_RB(9) AHV_RB(10) AHV_RB(11) AHV_RB(12) AHV_RB(13) AHV_RB(14) AHV_RB(15)
#undef AHV_RB
    default: return 0u;
  }
}

// Creation-order sum over one 16-edge chunk: `key` = the lane's edge vouchee, or
// 0xff when the edge is dead or absent; (lo, hi) = its bond's words.
__device__ __forceinline__ double chunk_sum(uint32_t key, uint32_t lo, uint32_t hi, uint32_t j, double acc) {
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const uint32_t k = row_bcast(key, u);
    const double b = __hiloint2double(static_cast<int>(row_bcast(hi, u)), static_cast<int>(row_bcast(lo, u)));
    const double t = acc + b;
    acc = k == j ? t : acc;
  }
  return acc;
}

__device__ __forceinline__ void stream_edge(const VouchCsrArgs& a, int32_t e, int32_t end, uint32_t& key, double& bd) {
  key = 0xffu;
  bd = 0.0;
  if (e < end) {
    bd = a.bonded[e];
    const uint32_t ve = a.vouchee[e];  // loaded with the liveness words, not after them
    key = live_edge(a.active, a.expiry_us, e, a.now_us) ? ve : 0xffu;
  }
}

template <int kStreamSlices>
__global__ __launch_bounds__(64 * kStreamWaves) void sigma_stream_kernel(VouchCsrArgs a) {
  constexpr int kStreamSessions = 4 * kStreamSlices * kStreamWaves;  // per 256-thread block
  const int l = threadIdx.x & 63;
  const uint32_t j = static_cast<uint32_t>(l & 15);
  const int64_t s0 = static_cast<int64_t>(blockIdx.x) * kStreamSessions + (threadIdx.x >> 6) * 4 * kStreamSlices;
  int32_t lo[kStreamSlices], hi[kStreamSlices];
  double sig[kStreamSlices], om[kStreamSlices], bd[kStreamSlices];
  uint32_t key[kStreamSlices];
#pragma unroll
  for (int q = 0; q < kStreamSlices; ++q) {
    const int64_t s = s0 + 4 * q + (l >> 4);
    const bool in = s < a.sessions;
    lo[q] = in ? a.offsets[s] : 0;
    hi[q] = in ? a.offsets[s + 1] : 0;
    sig[q] = in ? a.sigma[s * kTile + j] : 0.0;
    om[q] = in ? a.omega[s] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < kStreamSlices; ++q) stream_edge(a, lo[q] + static_cast<int32_t>(j), hi[q], key[q], bd[q]);
#pragma unroll
  for (int q = 0; q < kStreamSlices; ++q) {
    double acc = chunk_sum(key[q], static_cast<uint32_t>(__double2loint(bd[q])),
                           static_cast<uint32_t>(__double2hiint(bd[q])), j, 0.0);
    for (int32_t c = lo[q] + 16; c < hi[q]; c += 16) {  // group-uniform: > 16 edges
      uint32_t k2;
      double b2;
      stream_edge(a, c + static_cast<int32_t>(j), hi[q], k2, b2);
      acc = chunk_sum(k2, static_cast<uint32_t>(__double2loint(b2)), static_cast<uint32_t>(__double2hiint(b2)), j, acc);
    }
    const int64_t s = s0 + 4 * q + (l >> 4);
    if (s < a.sessions) a.sigma_eff[s * kTile + j] = sigma_eff_combine(score_or_zero(sig[q]), om[q], acc);
  }
}
template <int K>
void launch_stream_k(const VouchCsrArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(sigma_stream_kernel<K>, grid1(a.sessions, 4 * K * kStreamWaves), dim3(64 * kStreamWaves), 0, st, a);
}
void launch_sigma_eff_stream(const VouchCsrArgs& a, hipStream_t st) {
  if (a.sessions <= 0) return;
  static const int slices = [] {  // sessions per wave / 4 (A/B: AHV_STREAM_SLICES = 1, 2, 4)
    const char* e = std::getenv("AHV_STREAM_SLICES");
    const int k = e ? std::atoi(e) : 1;  // measured: 1 (62 VGPRs, 8 waves/SIMD) beats 2 and 4
    return k == 2 || k == 4 ? k : 1;
  }();
  if (slices == 2) launch_stream_k<2>(a, st);
  else if (slices == 4) launch_stream_k<4>(a, st);
  else launch_stream_k<1>(a, st);
  check_hip(hipGetLastError(), "sigma_stream_kernel");
}

// ------------------------------------------------------------------ K07

AHV_HD void release_elem(const VouchCsrArgs& a, int64_t s) {
  int32_t n = 0;
  for (int32_t k = a.offsets[s]; k < a.offsets[s + 1]; ++k) {
    if (a.active[k]) {
      a.active[k] = 0;
      a.released_us[k] = a.now_us;
      ++n;
    }
  }
  a.released[s] = n;
}
__global__ void release_kernel(VouchCsrArgs a) {
  for (int64_t s = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; s < a.sessions;
       s += static_cast<int64_t>(gridDim.x) * blockDim.x)
    release_elem(a, s);
}
void launch_release(const VouchCsrArgs& a, hipStream_t st) {
  if (a.sessions <= 0) return;
  hipLaunchKernelGGL(release_kernel, grid1(a.sessions), dim3(kBlock), 0, st, a);
  check_hip(hipGetLastError(), "release_kernel");
}
void release_host(const VouchCsrArgs& a) { for (int64_t s = 0; s < a.sessions; ++s) release_elem(a, s); }

// ------------------------------------------------------------------ K05
// Requests of a session are admitted in order; admitted ones become live edges
// for the following requests.  Live adjacency as a 16×16 bit matrix held in four
// 64-bit words (row v occupies bits 16·(v mod 4) … of word v/4).

AHV_HD uint32_t adj_row(const uint64_t w[4], int v) {
  const uint64_t x = (v >> 2) == 0 ? w[0] : (v >> 2) == 1 ? w[1] : (v >> 2) == 2 ? w[2] : w[3];
  return static_cast<uint32_t>((x >> (16 * (v & 3))) & 0xffffu);
}
AHV_HD void adj_set(uint64_t w[4], int v, int e) {
  const uint64_t bit = 1ull << (16 * (v & 3) + e);
  if ((v >> 2) == 0) w[0] |= bit;
  else if ((v >> 2) == 1) w[1] |= bit;
  else if ((v >> 2) == 2) w[2] |= bit;
  else w[3] |= bit;
}

// Per-session admission, O(E + R·16): one pass over the live edges builds the
// adjacency bits and each voucher's running exposure (creation order); every
// request then reads its voucher's running sum and, when admitted, adds its bond
// to it — the same additions in the same order as rescanning edges and earlier
// admitted requests, so the exposure test is bit-identical to the reference's.
// `Ed` supplies edge k (global arrays or an LDS stage); `exp` is 16 doubles.
template <class Ed>
AHV_HD void vouch_admit_body(const VouchAdmitArgs& a, int64_t s, const Ed& ed, double* exp, int xs) {
  uint64_t adj[4] = {0, 0, 0, 0};
  for (int u = 0; u < kTile; ++u) exp[u * xs] = 0.0;
  for (int32_t k = a.e_offsets[s]; k < a.e_offsets[s + 1]; ++k) {
    if (!ed.live(k)) continue;
    const int v = ed.voucher(k);
    adj_set(adj, v, ed.vouchee(k));
    exp[v * xs] += ed.bonded(k);
  }
  for (int32_t q = a.r_offsets[s]; q < a.r_offsets[s + 1]; ++q) {
    const int v = a.r_voucher[q], e = a.r_vouchee[q];
    const double sig = a.r_sigma[q];
    uint8_t code = 0;
    double bonded = 0.0;
    if (v == e) {
      code = 1;
    } else if (sig < kMinVoucherSigma) {
      code = 2;
    } else {
      // cycle: voucher reachable from vouchee through live edges
      uint32_t reach = adj_row(adj, e), seen = 0;
      while (reach & ~seen) {
        const uint32_t fresh = reach & ~seen;
        seen |= fresh;
        for (int u = 0; u < kTile; ++u)
          if ((fresh >> u) & 1u) reach |= adj_row(adj, u);
      }
      if ((reach >> v) & 1u) {
        code = 3;
      } else {
        double pct = a.r_pct[q];
        pct = pct < 0.0 ? 0.0 : (pct > 1.0 ? 1.0 : pct);
        bonded = sig * pct;
        if (exp[v * xs] + bonded > sig * a.max_exposure) code = 4;
      }
    }
    a.code[q] = code;
    a.r_bonded[q] = code == 0 ? bonded : 0.0;
    if (code == 0) {
      adj_set(adj, v, e);
      exp[v * xs] += bonded;
    }
  }
}

struct AdmitGlobalEdges {
  const VouchAdmitArgs* a;
  AHV_HD bool live(int32_t k) const { return live_edge(a->e_active, a->e_expiry, k, a->now_us); }
  AHV_HD int voucher(int32_t k) const { return a->e_voucher[k]; }
  AHV_HD int vouchee(int32_t k) const { return a->e_vouchee[k]; }
  AHV_HD double bonded(int32_t k) const { return a->e_bonded[k]; }
};

AHV_HD void vouch_admit_session(const VouchAdmitArgs& a, int64_t s) {
  double exp[kTile];
  vouch_admit_body(a, s, AdmitGlobalEdges{&a}, exp, 1);
}

// Device: 64 sessions per block (one lane each).  The block's contiguous edge
// range is staged in LDS with coalesced loads — voucher·16 + vouchee with 0xff
// for a dead edge, and the bond — and every lane keeps its 16 running exposures
// in an LDS row (dynamic voucher index: LDS, not scratch).  Ranges larger than
// the stage read global memory.
constexpr int kAdmitSessions = 64;
constexpr int kAdmitLdsEdges = 1024;
constexpr int kAdmitExpStride = kAdmitSessions + 1;  // exp[v] of lane t at v·65 + t: consecutive lanes, distinct banks

struct AdmitLdsEdges {
  int32_t e0;
  const uint8_t* key;
  const double* bd;
  __device__ bool live(int32_t k) const { return key[k - e0] != 0xff; }
  __device__ int voucher(int32_t k) const { return key[k - e0] >> 4; }
  __device__ int vouchee(int32_t k) const { return key[k - e0] & 15; }
  __device__ double bonded(int32_t k) const { return bd[k - e0]; }
};

__global__ __launch_bounds__(kAdmitSessions) void vouch_admit_kernel(VouchAdmitArgs a) {
  __shared__ uint8_t s_key[kAdmitLdsEdges];
  __shared__ double s_bd[kAdmitLdsEdges];
  __shared__ double s_exp[kTile * kAdmitExpStride];
  const int t = threadIdx.x;
  const int64_t s0 = static_cast<int64_t>(blockIdx.x) * kAdmitSessions;
  const int64_t s1 = s0 + kAdmitSessions < a.sessions ? s0 + kAdmitSessions : a.sessions;
  const int64_t s = s0 + t;
  const int32_t e0 = a.e_offsets[s0], e1 = a.e_offsets[s1];
  double* exp = s_exp + t;
  if (e1 - e0 > kAdmitLdsEdges) {  // block-uniform
    if (s < s1) vouch_admit_body(a, s, AdmitGlobalEdges{&a}, exp, kAdmitExpStride);
    return;
  }
  for (int32_t k = e0 + t; k < e1; k += kAdmitSessions) {
    const bool live = live_edge(a.e_active, a.e_expiry, k, a.now_us);
    s_key[k - e0] = live ? static_cast<uint8_t>((a.e_voucher[k] << 4) | a.e_vouchee[k]) : 0xffu;
    s_bd[k - e0] = a.e_bonded[k];
  }
  __syncthreads();
  if (s < s1) vouch_admit_body(a, s, AdmitLdsEdges{e0, s_key, s_bd}, exp, kAdmitExpStride);
}
void launch_vouch_admit(const VouchAdmitArgs& a, hipStream_t st) {
  if (a.sessions <= 0) return;
  hipLaunchKernelGGL(vouch_admit_kernel, grid1(a.sessions, kAdmitSessions), dim3(kAdmitSessions), 0, st, a);
  check_hip(hipGetLastError(), "vouch_admit_kernel");
}
void vouch_admit_host(const VouchAdmitArgs& a) { for (int64_t s = 0; s < a.sessions; ++s) vouch_admit_session(a, s); }

// ------------------------------------------------------------------ K06
// Depth-first cascade exactly as SlashingEngine.slash recurses: clip every live
// voucher of the current vouchee in creation order (releasing the bond), then
// descend into clipped vouchers left below floor+0.01 that still have live
// vouchers, up to depth 2.  Clip records are written in reference history order
// of the *clips* (parent clips before the child slash's clips).

// Edge access for one session's CSR range.  The host twin (and blocks whose
// edge range does not fit LDS) read the global arrays; the LDS view serves the
// staged copy: voucher, vouchee and a precomputed `live` byte per edge.
struct GlobalEdges {
  const SlashArgs* a;
  AHV_HD int voucher(int32_t k) const { return a->voucher[k]; }
  AHV_HD int vouchee(int32_t k) const { return a->vouchee[k]; }
  AHV_HD bool live(int32_t k) const { return live_edge(a->active, a->expiry_us, k, a->now_us); }
  AHV_HD void release(int32_t k) const {
    a->active[k] = 0;
    a->released_us[k] = a->now_us;
  }
  // the cascade walk reads back its own (uncapped) walk bytes, indexed from the
  // session's first edge — independent of how many records the caller kept
  AHV_HD void note_clip(int32_t b, int32_t i, int v, bool cascade) const {
    a->clip_walk[b + i] = static_cast<uint8_t>(v | (cascade ? 0x80 : 0));
  }
  AHV_HD int clip_voucher(int32_t b, int32_t ci) const { return a->clip_walk[b + ci] & 0x7f; }
  AHV_HD bool clip_cascades(int32_t b, int32_t ci) const { return (a->clip_walk[b + ci] & 0x80) != 0; }
};

template <class Edges>
AHV_HD bool has_live_voucher(const Edges& ed, int32_t b, int32_t e, int who) {
  for (int32_t k = b; k < e; ++k)
    if (ed.vouchee(k) == who && ed.live(k)) return true;
  return false;
}

// `sc` is the session's 16 scores (global row or LDS row, stride `ss`).
// The recursion is one loop over scalar state: a pending slash (who, depth) is
// run, which pushes its frame (its clip range); the walk then takes the next
// clip of the top frame and, if that voucher cascades, makes it the pending
// slash.  (A lambda called from two sites made the compiler address the frame
// slots through a pointer — scratch memory on the device, ~2 µs per step.)
template <class Edges>
AHV_HD void slash_session_t(const SlashArgs& a, int64_t s, const Edges& ed, double* sc, int ss) {
  if (a.target[s] >= kTile) {  // no slash in this session (storm subsets)
    a.clip_count[s] = 0;
    return;
  }
  const int32_t b = a.offsets[s], e = a.offsets[s + 1];
  const double omega = a.omega[s];
  const int32_t base = a.clip_offsets[s];
  int32_t nclip = 0;
  // explicit DFS stack, depth ≤ kMaxCascadeDepth (= 2): scalar slots, no arrays
  static_assert(kMaxCascadeDepth == 2, "scalar DFS frames assume a cascade depth of 2");
  int32_t next0 = 0, end0 = 0, next1 = 0, end1 = 0;
  int sp = 0;
  int who = a.target[s], who_depth = 0;
  bool pending = true;
  for (;;) {
    if (pending) {
      pending = false;
      sc[who * ss] = 0.0;
      const int32_t first = nclip;
      for (int32_t k = b; k < e; ++k) {
        if (ed.vouchee(k) != who || !ed.live(k)) continue;
        const int v = ed.voucher(k);
        const double x = sc[v * ss];
        const double before = x != x ? 0.0 : x;  // NaN = absent from agent_scores → 0.0
        const double after = clip_sigma(before, omega);
        sc[v * ss] = after;
        ed.note_clip(b, nclip, v, after < kCascadeBelow);
        if (nclip < a.clip_cap) {
          a.clip_voucher[base + nclip] = static_cast<uint8_t>(v);
          a.clip_depth[base + nclip] = static_cast<uint8_t>(who_depth);
          a.clip_before[base + nclip] = before;
          a.clip_after[base + nclip] = after;
        }
        ++nclip;
        ed.release(k);
      }
      // push the frame (a depth-2 frame never expands, so it needs no cursor)
      if (who_depth == 0) {
        next0 = first;
        end0 = nclip;
      } else if (who_depth == 1) {
        next1 = first;
        end1 = nclip;
      }
      sp = who_depth + 1;
    }
    if (sp == 0) break;
    const int depth = sp - 1;
    const int32_t nx = depth == 0 ? next0 : next1;
    const int32_t en = depth == 0 ? end0 : end1;
    if (depth >= kMaxCascadeDepth || nx >= en) {
      --sp;
      continue;
    }
    if (depth == 0) next0 = nx + 1;
    else next1 = nx + 1;
    const int v = ed.clip_voucher(b, nx);
    if (ed.clip_cascades(b, nx) && has_live_voucher(ed, b, e, v)) {
      who = v;
      who_depth = depth + 1;
      pending = true;
    }
  }
  a.clip_count[s] = nclip;
}

AHV_HD void slash_session(const SlashArgs& a, int64_t s) {
  slash_session_t(a, s, GlobalEdges{&a}, a.scores + s * kTile, 1);
}

// Fused K03 tail: σ_eff of vouchee j of session s over the post-slash live bonds
// (creation order — the sigma_eff_csr_elem sum).
AHV_HD double slash_sigma_eff(const SlashArgs& a, int64_t s, int j) {
  double contrib = 0.0;
  for (int32_t k = a.offsets[s]; k < a.offsets[s + 1]; ++k)
    if (a.vouchee[k] == j && live_edge(a.active, a.expiry_us, k, a.now_us)) contrib += a.bonded[k];
  return sigma_eff_combine(score_or_zero(a.scores[s * kTile + j]), a.omega[s], contrib);
}
AHV_HD void slash_sigma_row(const SlashArgs& a, int64_t s) {
  for (int j = 0; j < kTile; ++j) a.sigma_eff[s * kTile + j] = slash_sigma_eff(a, s, j);
}

// Device: a workgroup of 64 sessions stages its contiguous edge range
// (voucher, vouchee, live) and its 64×16 score rows in LDS with coalesced loads,
// runs the cascades out of LDS (one lane per session), and writes the scores
// back coalesced.  Releases go straight to global (sparse).  A block whose edge
// range exceeds the staging buffer falls back to the global-memory path.
constexpr int kSlashLdsEdges = 2048;
constexpr int kScorePad = kTile + 1;  // 17 doubles per row: spreads a column over banks
constexpr int kSlashClipLds = 16;    // clip records per lane cached in LDS
constexpr int kClipPad = kSlashClipLds + 4;

// (A 4-byte pad per 16 staged edges removes the 21 % LDS conflict cycles but
// costs a workgroup per CU of occupancy: measured 454 → 515 µs, so not used.)
__device__ __forceinline__ int32_t pad16(int32_t i) { return i; }
constexpr int kSlashLdsBytes = kSlashLdsEdges;

struct LdsEdges {
  const SlashArgs* a;
  int32_t e0;
  const uint8_t* vr;
  const uint8_t* ve;
  uint8_t* lv;
  __device__ int voucher(int32_t k) const { return vr[pad16(k - e0)]; }
  __device__ int vouchee(int32_t k) const { return ve[pad16(k - e0)]; }
  __device__ bool live(int32_t k) const { return lv[pad16(k - e0)] != 0; }
  __device__ void release(int32_t k) const {
    lv[pad16(k - e0)] = 0;
    a->active[k] = 0;
    a->released_us[k] = a->now_us;
  }
  // This lane's first kSlashClipLds clip records as (voucher | cascade<<7) bytes
  // in LDS: the cascade walk reads them back instead of waiting on a global
  // read-after-write of its own records (~2 µs per step of the walk).
  uint8_t* cl;
  __device__ void note_clip(int32_t b, int32_t i, int v, bool cascade) const {
    const uint8_t w = static_cast<uint8_t>(v | (cascade ? 0x80 : 0));
    if (i < kSlashClipLds) cl[i] = w;
    else a->clip_walk[b + i] = w;  // beyond the LDS cache: the uncapped global walk bytes
  }
  __device__ int clip_voucher(int32_t b, int32_t ci) const {
    return (ci < kSlashClipLds ? cl[ci] : a->clip_walk[b + ci]) & 0x7f;
  }
  __device__ bool clip_cascades(int32_t b, int32_t ci) const {
    return ((ci < kSlashClipLds ? cl[ci] : a->clip_walk[b + ci]) & 0x80) != 0;
  }
};

__global__ __launch_bounds__(64) void slash_kernel(SlashArgs a) {
  __shared__ uint8_t s_vr[kSlashLdsBytes], s_ve[kSlashLdsBytes], s_lv[kSlashLdsBytes];
  __shared__ double s_sc[64 * kScorePad];
  __shared__ uint8_t s_cl[64 * kClipPad];
  const int64_t s0 = static_cast<int64_t>(blockIdx.x) * 64;
  const int64_t s1 = s0 + 64 < a.sessions ? s0 + 64 : a.sessions;
  const int64_t s = s0 + threadIdx.x;
  const int32_t e0 = a.offsets[s0], e1 = a.offsets[s1];
  if (e1 - e0 > kSlashLdsEdges) {  // uniform per block
    if (s < a.sessions) slash_session(a, s);
    return;
  }
  for (int32_t k = e0 + threadIdx.x; k < e1; k += 64) {
    const int32_t j = pad16(k - e0);
    s_vr[j] = a.voucher[k];
    s_ve[j] = a.vouchee[k];
    s_lv[j] = live_edge(a.active, a.expiry_us, k, a.now_us) ? 1 : 0;
  }
  const int64_t nsc = (s1 - s0) * kTile;
  for (int64_t j = threadIdx.x; j < nsc; j += 64) s_sc[(j / kTile) * kScorePad + j % kTile] = a.scores[s0 * kTile + j];
  __syncthreads();
  if (s < a.sessions) slash_session_t(a, s, LdsEdges{&a, e0, s_vr, s_ve, s_lv, s_cl + threadIdx.x * kClipPad}, s_sc + threadIdx.x * kScorePad, 1);
  __syncthreads();
  for (int64_t j = threadIdx.x; j < nsc; j += 64) a.scores[s0 * kTile + j] = s_sc[(j / kTile) * kScorePad + j % kTile];
}

// σ_eff tail of the per-lane form (AHV_SLASH_PER_LANE), one thread per (session, vouchee).
__global__ void slash_sigma_kernel(SlashArgs a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < a.sessions * kTile) a.sigma_eff[i] = slash_sigma_eff(a, i / kTile, static_cast<int>(i % kTile));
}

// Group-cooperative form: 16 lanes per session (4 sessions per wave, 16 per
// 256-thread block).  Lane j holds edges j, j+16, j+32, j+48 of its session in
// registers (voucher, vouchee, live) and the session's score σ[j]; "which live
// edges vouch for `who`" is one ballot per 16 edges instead of a serial scan,
// and clips walk the ballot's set bits in edge (= creation) order, reading the
// voucher and its current σ with lane shuffles — the same clips, in the same
// order, with the same fp64 arithmetic as slash_session_t.  The cascade walk
// reads the group's clip list from LDS.  Sessions with more than
// kGroupEdges edges fall back to the one-lane global-memory form.
constexpr int kWaveLanes = 64;
constexpr int kSlashGroup = 16;
constexpr int kGroupChunks = 4;
constexpr int kGroupEdges = kSlashGroup * kGroupChunks;  // 64
constexpr int kSlashGroupsPerBlock = 16;

// σ_eff of the lane's vouchee j over the group's live edges, summed in edge
// (= creation) order: edge c·16 + k sits in lane k of chunk c; its vouchee (−1
// when dead) and bond arrive by lane shuffle, so all 16 lanes walk the same
// sequence and each adds the bonds of its own vouchee — the additions, in the
// order, of sigma_eff_csr_elem.
__device__ __forceinline__ double group_sigma_eff(const int (&ve)[kGroupChunks], const bool (&lv)[kGroupChunks],
                                                  const double (&bd)[kGroupChunks], int32_t n, int j, int gl0,
                                                  double sc, double omega) {
  double contrib = 0.0;
#pragma unroll
  for (int c = 0; c < kGroupChunks; ++c) {
    if (!__any(c * kSlashGroup < n)) break;
    const int vk_own = lv[c] ? ve[c] : -1;
#pragma unroll
    for (int k = 0; k < kSlashGroup; ++k) {
      const int vk = __shfl(vk_own, gl0 + k, kWaveLanes);
      const double bk = __shfl(bd[c], gl0 + k, kWaveLanes);
      if (vk == j) contrib += bk;
    }
  }
  return sigma_eff_combine(score_or_zero(sc), omega, contrib);
}

// The cascade of one slashed session on its 16-lane group (the edges already in
// registers: lane j holds edges j, j+16, j+32, j+48): ballots pick the live
// edges vouching for `who` in creation order, clips read the voucher and its σ by
// lane shuffle, the walk reads the group's clip list from LDS (`cl`).  Writes the
// session's scores row, clip records and count; returns the lane's final σ and
// leaves the released edges dead in `lv`.
__device__ __forceinline__ double group_cascade(const SlashArgs& a, int64_t s, int tgt, int32_t b, int j, int gl0,
                                                uint8_t* cl, const int (&vr)[kGroupChunks],
                                                const int (&ve)[kGroupChunks], bool (&lv)[kGroupChunks], double sc,
                                                double omega, int32_t* nclip_out = nullptr) {
  auto group_bits = [&](bool p) -> uint32_t {
    return static_cast<uint32_t>((__ballot(p) >> gl0) & 0xffffu);
  };
  const int32_t base = a.clip_offsets[s];
  int32_t nclip = 0;
  static_assert(kMaxCascadeDepth == 2, "scalar DFS frames assume a cascade depth of 2");
  int32_t next0 = 0, end0 = 0, next1 = 0, end1 = 0;
  int sp = 0;
  int who = tgt, who_depth = 0;
  bool pending = true;
  for (;;) {
    if (pending) {
      pending = false;
      if (j == who) sc = 0.0;
      const int32_t first = nclip;
#pragma unroll
      for (int c = 0; c < kGroupChunks; ++c) {
        uint32_t m = group_bits(ve[c] == who && lv[c]);
        while (m) {
          const int k = __builtin_ctz(m);
          m &= m - 1;
          const int v = __shfl(vr[c], gl0 + k, kWaveLanes);
          const double x = __shfl(sc, gl0 + v, kWaveLanes);
          const double before = x != x ? 0.0 : x;  // NaN = absent from agent_scores → 0.0
          const double after = clip_sigma(before, omega);
          if (j == v) sc = after;
          if (j == 0) {
            if (nclip < kGroupEdges) cl[nclip] = static_cast<uint8_t>(v | (after < kCascadeBelow ? 0x80 : 0));
            if (nclip < a.clip_cap) {
              a.clip_voucher[base + nclip] = static_cast<uint8_t>(v);
              a.clip_depth[base + nclip] = static_cast<uint8_t>(who_depth);
              a.clip_before[base + nclip] = before;
              a.clip_after[base + nclip] = after;
            }
          }
          if (j == k) {
            lv[c] = false;
            a.active[b + c * kSlashGroup + k] = 0;
            a.released_us[b + c * kSlashGroup + k] = a.now_us;
          }
          ++nclip;
        }
      }
      if (who_depth == 0) {
        next0 = first;
        end0 = nclip;
      } else if (who_depth == 1) {
        next1 = first;
        end1 = nclip;
      }
      sp = who_depth + 1;
    }
    if (sp == 0) break;
    const int depth = sp - 1;
    const int32_t nx = depth == 0 ? next0 : next1;
    const int32_t en = depth == 0 ? end0 : end1;
    if (depth >= kMaxCascadeDepth || nx >= en) {
      --sp;
      continue;
    }
    if (depth == 0) next0 = nx + 1;
    else next1 = nx + 1;
    const int c8 = cl[nx];  // every clip is cached: a group's session has ≤ kGroupEdges edges ≥ clips  // the LDS write by the group's lane 0 is visible: same wave
    const int v = c8 & 0x7f;
    if (!(c8 & 0x80)) continue;
    bool any_live = false;
#pragma unroll
    for (int c = 0; c < kGroupChunks; ++c) any_live = any_live || group_bits(ve[c] == v && lv[c]) != 0u;
    if (any_live) {
      who = v;
      who_depth = depth + 1;
      pending = true;
    }
  }
  a.scores[s * kTile + j] = sc;
  if (j == 0) a.clip_count[s] = nclip;
  if (nclip_out) *nclip_out = nclip;
  return sc;
}

__global__ __launch_bounds__(kSlashGroup * kSlashGroupsPerBlock) void slash_group_kernel(SlashArgs a) {
  __shared__ uint8_t s_cl[kSlashGroupsPerBlock][kGroupEdges];
  const int g = threadIdx.x / kSlashGroup;       // group in block
  const int j = threadIdx.x % kSlashGroup;       // lane in group
  const int gw = (threadIdx.x % kWaveLanes) / kSlashGroup;  // group in wave
  const int gl0 = gw * kSlashGroup;              // first wave lane of the group
  const int64_t s = static_cast<int64_t>(blockIdx.x) * kSlashGroupsPerBlock + g;
  if (s >= a.sessions) return;
  // target and edge range in one memory round trip (the range is 8 bytes per
  // session; the score row, 128 bytes, is only read for slashed sessions)
  const uint8_t tgt = a.target[s];
  const int32_t b = a.offsets[s], e = a.offsets[s + 1], n = e - b;
  const bool fused = a.sigma_eff != nullptr;
  if (tgt >= kTile && !fused) {  // group-uniform: no slash in this session
    if (j == 0) a.clip_count[s] = 0;
    return;
  }
  if (n > kGroupEdges) {
    if (j == 0) {
      slash_session(a, s);
      if (fused) slash_sigma_row(a, s);
    }
    return;
  }
  int vr[kGroupChunks], ve[kGroupChunks];
  bool lv[kGroupChunks];
  double bd[kGroupChunks];
#pragma unroll
  for (int c = 0; c < kGroupChunks; ++c) {
    const int32_t i = c * kSlashGroup + j;
    const bool in = i < n;
    vr[c] = in && tgt < kTile ? a.voucher[b + i] : 0;
    ve[c] = in ? a.vouchee[b + i] : -1;
    lv[c] = in && live_edge(a.active, a.expiry_us, b + i, a.now_us);
    bd[c] = in && fused ? a.bonded[b + i] : 0.0;
  }
  double sc = a.scores[s * kTile + j];
  const double omega = a.omega[s];
  if (tgt >= kTile) {  // fused, no slash here: σ_eff only
    if (j == 0) a.clip_count[s] = 0;
    a.sigma_eff[s * kTile + j] = group_sigma_eff(ve, lv, bd, n, j, gl0, sc, omega);
    return;
  }
  sc = group_cascade(a, s, tgt, b, j, gl0, s_cl[g], vr, ve, lv, sc, omega);
  if (fused) a.sigma_eff[s * kTile + j] = group_sigma_eff(ve, lv, bd, n, j, gl0, sc, omega);
}

// Split form (default): the cascade runs over the slashed sessions only and the
// σ_eff of every session is the streaming K03 pass afterwards.
//
// Cascade: a wave scans 64 sessions (targets + edge ranges in one coalesced
// round trip, clip_count 0 for the untouched ones), takes the slashed ones in
// batches of kWaveBatch — loading every edge of the batch at once, lane l =
// edge l of a session (≤ 64 edges), and the score rows — and then runs each
// cascade with the whole wave on one session.  The walk's state is
// wave-uniform, so "which live edges vouch for `who`" is one 64-bit ballot and
// every read of another lane's value (the clipped voucher, its σ, the clip list)
// is a v_readlane into an SGPR — a few cycles, where the 16-lane group form
// pays an LDS-crossbar ds_bpermute round trip per read on the cascade's
// critical path.  The clip list lives one entry per lane in a VGPR.  Clip
// order, arithmetic and records are those of slash_session_t.
constexpr int kWaveBatch = 8;  // slashed sessions loaded per round trip

__device__ __forceinline__ int rl_i(int x, int lane) { return __builtin_amdgcn_readlane(x, lane); }
__device__ __forceinline__ double rl_d(double x, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
  return __hiloint2double(hi, lo);
}

// One slashed session on the whole wave: lane l holds edge l (`e8` = voucher |
// vouchee << 8, 0xffff when absent; `live`), lanes 0..15 its σ row.
__device__ __forceinline__ void wave_cascade(const SlashArgs& a, int64_t s, int tgt, int32_t b, int l,
                                             uint32_t e8, bool live, double sc, double omega) {
  const int vr = static_cast<int>(e8 & 0xffu), ve = static_cast<int>((e8 >> 8) & 0xffu);
  const int32_t base = a.clip_offsets[s];
  uint32_t clv = 0;  // clip list: lane i = clip i as (voucher | cascade << 7)
  int32_t nclip = 0;
  static_assert(kMaxCascadeDepth == 2, "scalar DFS frames assume a cascade depth of 2");
  int32_t next0 = 0, end0 = 0, next1 = 0, end1 = 0;
  int sp = 0;
  int who = tgt, who_depth = 0;
  bool pending = true;
  for (;;) {
    if (pending) {
      pending = false;
      if (l == who) sc = 0.0;
      const int32_t first = nclip;
      uint64_t m = __ballot(ve == who && live);
      while (m) {
        const int k = static_cast<int>(__builtin_ctzll(m));
        m &= m - 1;
        const int v = rl_i(vr, k);
        const double x = rl_d(sc, v);
        const double before = x != x ? 0.0 : x;  // NaN = absent from agent_scores → 0.0
        const double after = clip_sigma(before, omega);
        if (l == v) sc = after;
        if (l == nclip) clv = static_cast<uint32_t>(v | (after < kCascadeBelow ? 0x80 : 0));
        if (l == 0 && nclip < a.clip_cap) {
          a.clip_voucher[base + nclip] = static_cast<uint8_t>(v);
          a.clip_depth[base + nclip] = static_cast<uint8_t>(who_depth);
          a.clip_before[base + nclip] = before;
          a.clip_after[base + nclip] = after;
        }
        if (l == k) {
          live = false;
          a.active[b + k] = 0;
          a.released_us[b + k] = a.now_us;
        }
        ++nclip;
      }
      if (who_depth == 0) {
        next0 = first;
        end0 = nclip;
      } else if (who_depth == 1) {
        next1 = first;
        end1 = nclip;
      }
      sp = who_depth + 1;
    }
    if (sp == 0) break;
    const int depth = sp - 1;
    const int32_t nx = depth == 0 ? next0 : next1;
    const int32_t en = depth == 0 ? end0 : end1;
    if (depth >= kMaxCascadeDepth || nx >= en) {
      --sp;
      continue;
    }
    if (depth == 0) next0 = nx + 1;
    else next1 = nx + 1;
    const int c8 = rl_i(static_cast<int>(clv), nx);
    const int v = c8 & 0x7f;
    if ((c8 & 0x80) && __ballot(ve == v && live) != 0ull) {
      who = v;
      who_depth = depth + 1;
      pending = true;
    }
  }
  if (l < kTile) a.scores[s * kTile + l] = sc;
  if (l == 0) a.clip_count[s] = nclip;
}

__global__ __launch_bounds__(256) void slash_wave_kernel(SlashArgs a) {
  const int l = threadIdx.x & 63;
  const int64_t w0 = (static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6)) * kWaveLanes;
  if (w0 >= a.sessions) return;  // wave-uniform
  const int64_t s_me = w0 + l;
  const bool in = s_me < a.sessions;
  const uint8_t tg = in ? a.target[s_me] : 0xff;
  const int32_t off0 = a.offsets[in ? s_me : a.sessions];
  const int32_t off1 = a.offsets[in ? s_me + 1 : a.sessions];
  const bool hit = tg < kTile;
  if (in && !hit) a.clip_count[s_me] = 0;
  uint64_t m = __ballot(hit);
  while (m) {  // wave-uniform
    int idx[kWaveBatch];
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < kWaveBatch; ++i) {
      idx[i] = m ? static_cast<int>(__builtin_ctzll(m)) : 0;
      cnt += m ? 1 : 0;
      m &= m ? m - 1 : 0ull;
    }
    uint32_t e8[kWaveBatch];
    bool live[kWaveBatch];
    double sc[kWaveBatch], om[kWaveBatch];
#pragma unroll
    for (int i = 0; i < kWaveBatch; ++i) {  // every load of the batch in flight at once
      const int32_t b = rl_i(off0, idx[i]), n = rl_i(off1, idx[i]) - b;
      const bool use = i < cnt && n <= kWaveLanes;
      const bool mine = use && l < n;
      e8[i] = mine ? (static_cast<uint32_t>(a.voucher[b + l]) | (static_cast<uint32_t>(a.vouchee[b + l]) << 8))
                   : 0xffffu;
      live[i] = mine && live_edge(a.active, a.expiry_us, b + l, a.now_us);
      sc[i] = use && l < kTile ? a.scores[(w0 + idx[i]) * kTile + l] : 0.0;
      om[i] = i < cnt ? a.omega[w0 + idx[i]] : 0.0;
    }
#pragma unroll 1
    for (int i = 0; i < cnt; ++i) {  // one copy of the cascade code: the batch rotates through slot 0
      const int64_t s = w0 + idx[0];
      const int32_t b = rl_i(off0, idx[0]), n = rl_i(off1, idx[0]) - b;
      if (n > kWaveLanes) {  // more edges than lanes: the one-lane global-memory form
        if (l == 0) slash_session(a, s);
      } else {
        wave_cascade(a, s, rl_i(static_cast<int>(tg), idx[0]), b, l, e8[0], live[0], sc[0], om[0]);
      }
#pragma unroll
      for (int j = 0; j + 1 < kWaveBatch; ++j) {
        idx[j] = idx[j + 1];
        e8[j] = e8[j + 1];
        live[j] = live[j + 1];
        sc[j] = sc[j + 1];
        om[j] = om[j + 1];
      }
    }
  }
}

// Default split cascade: a 256-thread block owns a window of 256 sessions.  One
// coalesced round trip reads the window's targets and edge offsets (offsets
// into LDS; clip_count 0 for the untouched), wave ballots + a 4-entry prefix
// compact the slashed ones into an LDS list, and the 16 groups of 16 lanes take
// the list round-robin: a group requests its session's edges (lane j: edges
// j, j+16, j+32, j+48 — one round trip, liveness words included), σ row and ω,
// then runs group_cascade.  (slash_wave_kernel — one session per wave with
// v_readlane instead of ds_bpermute — issues far fewer LDS ops but serialises
// ~6 sessions per wave on SALU: slower, kept for A/B as mode 3.)
constexpr int kCascWindow = 256;

__global__ __launch_bounds__(kCascWindow) void slash_cascade_kernel(SlashArgs a) {
  __shared__ int32_t s_list[kCascWindow];
  __shared__ int32_t s_off[kCascWindow + 1];
  __shared__ int32_t s_wcount[kCascWindow / kWaveLanes];
  __shared__ uint8_t s_cl[kSlashGroupsPerBlock][kGroupEdges];
  __shared__ int32_t s_nclip[kCascWindow];
  const int t = threadIdx.x;
  const int w = t / kWaveLanes, l = t % kWaveLanes;
  const int64_t w0 = static_cast<int64_t>(blockIdx.x) * kCascWindow;
  const int64_t s_me = w0 + t;
  const bool in_range = s_me < a.sessions;
  const uint8_t tg = in_range ? a.target[s_me] : 0xff;
  s_off[t] = a.offsets[in_range ? s_me : a.sessions];
  if (t == kCascWindow - 1) s_off[kCascWindow] = a.offsets[s_me + 1 < a.sessions ? s_me + 1 : a.sessions];
  const bool hit = tg < kTile;
  if (in_range && !hit) a.clip_count[s_me] = 0;
  const uint64_t m = __ballot(hit);
  if (l == 0) s_wcount[w] = __popcll(m);
  __syncthreads();
  int pre = 0, total = 0;
#pragma unroll
  for (int k = 0; k < kCascWindow / kWaveLanes; ++k) {
    pre += k < w ? s_wcount[k] : 0;
    total += s_wcount[k];
  }
  if (hit) s_list[pre + __popcll(m & ((1ull << l) - 1ull))] = t | (static_cast<int>(tg) << 16);
  __syncthreads();
  const int g = t / kSlashGroup, j = t % kSlashGroup;
  const int gl0 = (t % kWaveLanes) / kSlashGroup * kSlashGroup;
  for (int idx = g; idx < total; idx += kSlashGroupsPerBlock) {  // group-uniform
    const int e = s_list[idx];
    const int ls = e & 0xffff, tgt = e >> 16;
    const int64_t s = w0 + ls;
    const int32_t b = s_off[ls], n = s_off[ls + 1] - b;
    if (n > kGroupEdges) {  // beyond the registers: the one-lane global-memory form
      if (j == 0) {
        slash_session(a, s);
        s_nclip[ls] = a.clip_count[s];  // this thread's own write
      }
      continue;
    }
    int vr[kGroupChunks], ve[kGroupChunks];
    bool lv[kGroupChunks];
#pragma unroll
    for (int c = 0; c < kGroupChunks; ++c) {
      const int32_t i = c * kSlashGroup + j;
      const bool in = i < n;
      vr[c] = in ? a.voucher[b + i] : 0;
      ve[c] = in ? a.vouchee[b + i] : -1;
      lv[c] = in && live_edge(a.active, a.expiry_us, b + i, a.now_us);
    }
    const double sc = a.scores[s * kTile + j];
    int32_t nclip = 0;
    group_cascade(a, s, tgt, b, j, gl0, s_cl[g], vr, ve, lv, sc, a.omega[s], &nclip);
    if (j == 0) s_nclip[ls] = nclip;
  }
  if (a.touched_tmp == nullptr) return;  // block-uniform
  // touched sessions (≥ 1 clip) of the window, in session order: per-wave ballots
  // + prefix into a window-local segment; touched_compact places the segments
  __syncthreads();
  const bool touched = hit && s_nclip[t] > 0;
  const uint64_t tm = __ballot(touched);
  if (l == 0) s_wcount[w] = __popcll(tm);
  __syncthreads();
  int tpre = 0, ttotal = 0;
#pragma unroll
  for (int k = 0; k < kCascWindow / kWaveLanes; ++k) {
    tpre += k < w ? s_wcount[k] : 0;
    ttotal += s_wcount[k];
  }
  if (touched) a.touched_tmp[w0 + tpre + __popcll(tm & ((1ull << l) - 1ull))] = static_cast<int32_t>(s_me);
  if (t == 0) a.touched_blocks[blockIdx.x] = ttotal;
}

// Window segments of the touched list from clip_count (the non-split forms).
__global__ __launch_bounds__(kCascWindow) void touched_flags_kernel(SlashArgs a) {
  __shared__ int32_t s_wcount[kCascWindow / kWaveLanes];
  const int t = threadIdx.x, w = t / kWaveLanes, l = t % kWaveLanes;
  const int64_t w0 = static_cast<int64_t>(blockIdx.x) * kCascWindow, s_me = w0 + t;
  const bool touched = s_me < a.sessions && a.clip_count[s_me] > 0;
  const uint64_t tm = __ballot(touched);
  if (l == 0) s_wcount[w] = __popcll(tm);
  __syncthreads();
  int tpre = 0, ttotal = 0;
#pragma unroll
  for (int k = 0; k < kCascWindow / kWaveLanes; ++k) {
    tpre += k < w ? s_wcount[k] : 0;
    ttotal += s_wcount[k];
  }
  if (touched) a.touched_tmp[w0 + tpre + __popcll(tm & ((1ull << l) - 1ull))] = static_cast<int32_t>(s_me);
  if (t == 0) a.touched_blocks[blockIdx.x] = ttotal;
}

// touched_compact: exclusive prefix of the per-window counts (one workgroup),
// then every window copies its segment to its offset — the touched list in
// session order without a device-wide sort or a host round trip per window.
__global__ __launch_bounds__(1024) void touched_scan_kernel(const int32_t* counts, int64_t nblocks, int32_t* offsets,
                                                            int64_t* total) {
  __shared__ int32_t s_sum[1024];
  __shared__ int32_t s_run;
  const int t = threadIdx.x;
  if (t == 0) s_run = 0;
  __syncthreads();
  for (int64_t base = 0; base < nblocks; base += 1024) {
    const int32_t c = base + t < nblocks ? counts[base + t] : 0;
    s_sum[t] = c;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // Hillis–Steele inclusive scan
      const int32_t y = t >= d ? s_sum[t - d] : 0;
      __syncthreads();
      s_sum[t] += y;
      __syncthreads();
    }
    if (base + t < nblocks) offsets[base + t] = s_run + s_sum[t] - c;
    __syncthreads();
    if (t == 0) s_run += s_sum[1023];
    __syncthreads();
  }
  if (t == 0) *total = s_run;
}

__global__ __launch_bounds__(kCascWindow) void touched_copy_kernel(const int32_t* counts, const int32_t* offsets,
                                                                   const int32_t* tmp, int64_t* out) {
  const int64_t blk = blockIdx.x;
  const int32_t c = counts[blk];
  if (static_cast<int32_t>(threadIdx.x) < c)
    out[offsets[blk] + threadIdx.x] = tmp[blk * kCascWindow + threadIdx.x];
}

void launch_slash(const SlashArgs& a, hipStream_t st) {
  if (a.sessions <= 0) return;
  static const bool per_lane = [] {
    const char* e = std::getenv("AHV_SLASH_PER_LANE");
    return e && std::atoi(e) == 1;
  }();
  static const int env_mode = [] {  // A/B: AHV_SLASH_FUSED=1 the round-2 single pass; AHV_SLASH_MODE=0..3
    const char* f = std::getenv("AHV_SLASH_FUSED");
    const char* m = std::getenv("AHV_SLASH_MODE");
    return f && std::atoi(f) == 1 ? 1 : m ? std::atoi(m) : 0;
  }();
  const int mode = a.mode >= 0 ? a.mode : (per_lane ? 2 : env_mode);
  if (mode == 2) {
    hipLaunchKernelGGL(slash_kernel, grid1(a.sessions, 64), dim3(64), 0, st, a);
    if (a.sigma_eff) hipLaunchKernelGGL(slash_sigma_kernel, grid1(a.sessions * kTile), dim3(kBlock), 0, st, a);
  } else if (mode == 1) {
    hipLaunchKernelGGL(slash_group_kernel, grid1(a.sessions, kSlashGroupsPerBlock),
                       dim3(kSlashGroup * kSlashGroupsPerBlock), 0, st, a);
  } else {
    if (mode == 3) hipLaunchKernelGGL(slash_wave_kernel, grid1(a.sessions, 4 * kWaveLanes), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(slash_cascade_kernel, grid1(a.sessions, kCascWindow), dim3(kCascWindow), 0, st, a);

    if (a.sigma_eff) {  // K03 over the post-slash scores and bonds
      static const bool csr = [] {  // A/B: AHV_SLASH_SIGMA=csr runs the LDS-staged K03 form
        const char* e = std::getenv("AHV_SLASH_SIGMA");
        return e && std::string(e) == "csr";
      }();
      const VouchCsrArgs v{a.sessions, a.now_us, a.offsets, a.voucher, a.vouchee, a.bonded, a.active,
                           a.expiry_us, a.released_us, nullptr, a.scores, a.omega, a.sigma_eff, nullptr};
      if (csr) launch_sigma_eff_csr(v, st);
      else launch_sigma_eff_stream(v, st);
    }
  }
  if (a.touched_tmp != nullptr) {  // the touched list (split mode: segments written by the cascade)
    const int64_t nb = (a.sessions + kCascWindow - 1) / kCascWindow;
    if (mode != 0) hipLaunchKernelGGL(touched_flags_kernel, dim3(static_cast<uint32_t>(nb)), dim3(kCascWindow), 0, st, a);
    hipLaunchKernelGGL(touched_scan_kernel, dim3(1), dim3(1024), 0, st, a.touched_blocks, nb, a.touched_offsets,
                       a.touched_total);
    hipLaunchKernelGGL(touched_copy_kernel, dim3(static_cast<uint32_t>(nb)), dim3(kCascWindow), 0, st,
                       a.touched_blocks, a.touched_offsets, a.touched_tmp, a.touched);
  }
  check_hip(hipGetLastError(), "slash_kernel");
}
void slash_host(const SlashArgs& a) {
  for (int64_t s = 0; s < a.sessions; ++s) {
    slash_session(a, s);
    if (a.sigma_eff) slash_sigma_row(a, s);
  }
  if (a.touched != nullptr) {
    int64_t n = 0;
    for (int64_t s = 0; s < a.sessions; ++s)
      if (a.clip_count[s] > 0) a.touched[n++] = s;
    *a.touched_total = n;
  }
}


void kernels_liability(std::vector<KernelEntry>& out) {
  out.push_back({"slash_group_kernel", reinterpret_cast<const void*>(&slash_group_kernel)});
  out.push_back({"slash_cascade_kernel", reinterpret_cast<const void*>(&slash_cascade_kernel)});
  out.push_back({"slash_wave_kernel", reinterpret_cast<const void*>(&slash_wave_kernel)});
  out.push_back({"sigma_stream_kernel<1>", reinterpret_cast<const void*>(&sigma_stream_kernel<1>)});
  out.push_back({"slash_kernel", reinterpret_cast<const void*>(&slash_kernel)});
  out.push_back({"sigma_eff_csr_kernel", reinterpret_cast<const void*>(&sigma_eff_csr_kernel)});
  out.push_back({"build_tiles_kernel", reinterpret_cast<const void*>(&build_tiles_kernel)});
  out.push_back({"bond_tiles_mfma_kernel", reinterpret_cast<const void*>(&bond_tiles_mfma_kernel)});
  out.push_back({"bond_fused_mfma_kernel", reinterpret_cast<const void*>(&bond_fused_mfma_kernel)});
  out.push_back({"vouch_admit_kernel", reinterpret_cast<const void*>(&vouch_admit_kernel)});
}

}  // namespace ahv
