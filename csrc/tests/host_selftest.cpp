// Host-side self test of the native core under AddressSanitizer and
// UndefinedBehaviorSanitizer.  It drives every kernel's host twin
// — the exact __host__ __device__ bodies the gfx950 kernels run — on random
// inputs of awkward sizes, plus the batched pipeline with a hand-built string
// pool, and checks internal consistency (SHA-256 vectors, fused vs step-loop
// sagas, MFMA-order vs creation-order σ_eff, Merkle of the pipeline's own
// digests).  Built and run by scripts/sanitize_host.sh; exits non-zero on any
// failed check (and the sanitizers abort on any memory or UB error).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "ahv/kernels.h"
#include "ahv/launch.h"
#include "ahv/pipeline.h"
#include "ahv/saga_batch.h"
#include "ahv/store_host.h"
#include "ahv/store_template.h"

using namespace ahv;

static int g_fail = 0;
#define CHECK(cond)                                                      \
  do {                                                                   \
    if (!(cond)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                          \
    }                                                                    \
  } while (0)

static std::mt19937_64 rng(1234);
static int rnd(int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); }
static double rndf() { return std::uniform_real_distribution<double>(0.0, 1.0)(rng); }

static std::string hex(const uint32_t* d) {
  char b[65];
  for (int k = 0; k < 8; ++k) std::snprintf(b + 8 * k, 9, "%08x", d[k]);
  return std::string(b, 64);
}

// ------------------------------------------------------------------ audit
static void test_hashing() {
  const std::vector<std::string> msgs = {"", "abc", std::string(55, 'x'), std::string(56, 'y'),
                                         std::string(64, 'z'), std::string(1000, 'q')};
  std::vector<uint8_t> arena;
  std::vector<int64_t> off{0};
  for (auto& m : msgs) {
    arena.insert(arena.end(), m.begin(), m.end());
    off.push_back(static_cast<int64_t>(arena.size()));
  }
  std::vector<uint32_t> dig(msgs.size() * 8);
  HashManyArgs h{static_cast<int64_t>(msgs.size()), arena.data(), off.data(), dig.data()};
  hash_many_host(h);
  CHECK(hex(&dig[0]) == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855");
  CHECK(hex(&dig[8]) == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad");

  // Merkle of 1 leaf is the leaf; of n random leaves runs for awkward n
  for (int n : {1, 2, 3, 5, 8, 13, 64, 65}) {
    std::vector<uint32_t> leaves(n * 8), scratch(n * 8), root(8);
    for (auto& w : leaves) w = static_cast<uint32_t>(rng());
    int32_t offs[2] = {0, n};
    MerkleArgs m{1, offs, leaves.data(), scratch.data(), root.data()};
    merkle_host(m);
    if (n == 1) CHECK(std::memcmp(root.data(), leaves.data(), 32) == 0);
  }
  // verify: recompute digests of the arena and check a 3-delta chain's links
  std::vector<uint32_t> parent(msgs.size() * 8, 0);
  std::vector<uint8_t> hp(msgs.size(), 0), dok(msgs.size()), cok(1);
  for (size_t i = 1; i < msgs.size(); ++i) {
    std::memcpy(&parent[i * 8], &dig[(i - 1) * 8], 32);
    hp[i] = 1;
  }
  int32_t coff[2] = {0, static_cast<int32_t>(msgs.size())};
  VerifyArgs v{static_cast<int64_t>(msgs.size()), 1, arena.data(), off.data(), dig.data(), parent.data(),
               hp.data(), coff, dok.data(), cok.data()};
  verify_host(v);
  CHECK(cok[0] == 1);
  // chain re-derivation over prefix/suffix records
  const std::string pre = "{\"a\": 1, \"parent_hash\": ", suf = ", \"z\": 2}";
  std::vector<uint8_t> ca(pre.begin(), pre.end());
  ca.insert(ca.end(), suf.begin(), suf.end());
  const int D = 7;
  std::vector<int64_t> po(D, 0), so(D, static_cast<int64_t>(pre.size()));
  std::vector<int32_t> pl(D, static_cast<int32_t>(pre.size())), sl(D, static_cast<int32_t>(suf.size()));
  std::vector<uint32_t> cd(D * 8);
  int32_t chain_off[3] = {0, 3, D};
  ChainHashArgs c{2, chain_off, ca.data(), po.data(), pl.data(), so.data(), sl.data(), nullptr, nullptr, cd.data()};
  chain_hash_host(c);
  CHECK(std::memcmp(&cd[0], &cd[3 * 8], 32) == 0);  // both chains start from `null`
}

// ------------------------------------------------------------------ sagas
static void test_sagas() {
  for (int K : {1, 3, 10, 16, 17, 24}) {
    const int S = 257;
    const size_t n = static_cast<size_t>(S) * K;
    std::vector<uint8_t> fa(n), fk(n), cf(n), hu(n), mr(n);
    for (size_t e = 0; e < n; ++e) {
      fa[e] = rndf() < 0.1 ? 255 : (rndf() < 0.1 ? 1 : 0);
      fk[e] = static_cast<uint8_t>(rnd(1, 2));
      cf[e] = rndf() < 0.2 ? static_cast<uint8_t>(rnd(1, 2)) : 0;
      hu[e] = rndf() < 0.9;
      mr[e] = static_cast<uint8_t>(rnd(0, 2));
    }
    struct Out {
      std::vector<uint8_t> st, rc, er, gs;
      std::vector<int64_t> t0, t1, gd;
      std::vector<int32_t> fs, cfc, tk;
      std::vector<unsigned long long> stats;
      Out(size_t n, int S)
          : st(n), rc(n), er(n), gs(S), t0(n), t1(n), gd(S), fs(S), cfc(S), tk(S), stats(4 * kStatSpread, 0) {}
      SagaBatchArgs args(int S, int K, const std::vector<uint8_t>* in[5]) {
        return SagaBatchArgs{S, K, 1, 1000, in[0]->data(), in[1]->data(), in[2]->data(), in[3]->data(),
                             in[4]->data(), st.data(), rc.data(), er.data(), t0.data(), t1.data(), gs.data(),
                             gd.data(), fs.data(), cfc.data(), tk.data(), stats.data()};
      }
    };
    const std::vector<uint8_t>* in[5] = {&fa, &fk, &cf, &hu, &mr};
    Out a(n, S), b(n, S);
    saga_fused_host(a.args(S, K, in));
    SagaBatchArgs bb = b.args(S, K, in);
    saga_phase_host(bb, 0, 0);
    for (int k = 0; k < K; ++k) saga_phase_host(bb, 1, k);
    saga_phase_host(bb, 2, 0);
    for (int k = K - 1; k >= 0; --k) saga_phase_host(bb, 3, k);
    saga_phase_host(bb, 4, 0);
    CHECK(a.st == b.st && a.rc == b.rc && a.er == b.er && a.t0 == b.t0 && a.t1 == b.t1);
    CHECK(a.gs == b.gs && a.gd == b.gd && a.fs == b.fs && a.cfc == b.cfc && a.tk == b.tk);
    CHECK(a.stats == b.stats);
  }
}

// -------------------------------------------------------------- liability
static void test_liability() {
  const int S = 97;
  std::vector<int32_t> off{0};
  std::vector<uint8_t> vr, ve, ac;
  std::vector<double> bd;
  std::vector<int64_t> ex, rel;
  for (int s = 0; s < S; ++s) {
    const int E = rnd(0, 40);
    for (int k = 0; k < E; ++k) {
      const int a = rnd(0, 15);
      vr.push_back(static_cast<uint8_t>(a));
      ve.push_back(static_cast<uint8_t>((a + rnd(1, 15)) % 16));
      bd.push_back(rndf() * 0.3);
      ac.push_back(rndf() < 0.9);
      ex.push_back(rndf() < 0.2 ? rnd(0, 200) : -1);
      rel.push_back(0);
    }
    off.push_back(static_cast<int32_t>(vr.size()));
  }
  std::vector<double> sigma(S * 16), omega(S), tiles(S * 256), se(S * 16), se2(S * 16), expo(S * 16), bin(S * 16);
  for (auto& x : sigma) x = rndf();
  for (auto& x : omega) x = rndf();
  VouchCsrArgs c{S, 100, off.data(), vr.data(), ve.data(), bd.data(), ac.data(), ex.data(), rel.data(),
                 tiles.data(), sigma.data(), omega.data(), se.data(), nullptr};
  build_tiles_host(c);
  sigma_eff_csr_host(c);
  BondTileArgs bt{S, tiles.data(), sigma.data(), omega.data(), se2.data(), expo.data(), bin.data()};
  bond_tiles_host(bt);
  for (int i = 0; i < S * 16; ++i) CHECK(std::fabs(se[i] - se2[i]) < 1e-12);
  // admission of random requests
  std::vector<int32_t> roff{0};
  std::vector<uint8_t> rv, re, code;
  std::vector<double> rs, rp, rb;
  for (int s = 0; s < S; ++s) {
    for (int q = rnd(0, 9); q > 0; --q) {
      rv.push_back(static_cast<uint8_t>(rnd(0, 15)));
      re.push_back(static_cast<uint8_t>(rnd(0, 15)));
      rs.push_back(rndf());
      rp.push_back(rndf());
    }
    roff.push_back(static_cast<int32_t>(rv.size()));
  }
  code.resize(rv.size());
  rb.resize(rv.size());
  VouchAdmitArgs va{S, 100, 0.8, off.data(), vr.data(), ve.data(), bd.data(), ac.data(), ex.data(), roff.data(),
                    rv.data(), re.data(), rs.data(), rp.data(), rb.data(), code.data()};
  vouch_admit_host(va);
  for (size_t q = 0; q < rv.size(); ++q) {
    CHECK(code[q] <= 4);
    if (rv[q] == re[q]) CHECK(code[q] == 1);
  }
  // slash cascade then release
  std::vector<uint8_t> tgt(S);
  for (auto& t : tgt) t = static_cast<uint8_t>(rnd(0, 15));
  std::vector<double> scores(S * 16);
  for (auto& x : scores) x = rndf() < 0.1 ? NAN : rndf();
  const int cap = 8;  // deliberately small: overflowing clip records must stay in bounds
  std::vector<int32_t> coffs(S), ccount(S);
  for (int s = 0; s < S; ++s) coffs[s] = s * cap;
  std::vector<uint8_t> cv(S * cap), cd(S * cap);
  std::vector<double> cb(S * cap), ca(S * cap);
  SlashArgs sa{S, 100, off.data(), vr.data(), ve.data(), ac.data(), ex.data(), rel.data(), tgt.data(),
               omega.data(), scores.data(), coffs.data(), ccount.data(), cv.data(), cd.data(), cb.data(), ca.data(),
               cap};
  std::vector<uint8_t> walk(std::max<size_t>(vr.size(), 1));  // the cascade's uncapped walk bytes
  sa.clip_walk = walk.data();
  slash_host(sa);
  // the violator is zeroed; a vouch cycle back to it can re-clip it to the floor
  for (int s = 0; s < S; ++s) CHECK(scores[s * 16 + tgt[s]] == 0.0 || scores[s * 16 + tgt[s]] == kSigmaFloor);
  std::vector<int32_t> released(S);
  VouchCsrArgs r = c;
  r.released = released.data();
  release_host(r);
  for (auto a : ac) CHECK(a == 0);
}

// ------------------------------------------------------------- governance
static void test_governance() {
  const int n = 1001;
  std::vector<double> sigma(n);
  std::vector<uint8_t> cons(n), ring(n), flags(n), wit(n), req(n), reason(n);
  for (int i = 0; i < n; ++i) {
    sigma[i] = rndf();
    cons[i] = rnd(0, 1);
    flags[i] = static_cast<uint8_t>(rnd(0, 7));
    wit[i] = rnd(0, 1);
  }
  RingGateArgs g{n, sigma.data(), cons.data(), ring.data()};
  ring_gate_host(g);
  RingCheckArgs rc{n, ring.data(), flags.data(), sigma.data(), cons.data(), wit.data(), req.data(), reason.data()};
  ring_check_host(rc);
  std::vector<uint8_t> st(n), tg(n), ok(n);
  std::vector<int64_t> t0(n), t1(n);
  for (int i = 0; i < n; ++i) {
    st[i] = static_cast<uint8_t>(rnd(0, 6));
    tg[i] = static_cast<uint8_t>(rnd(0, 9));  // includes out-of-range targets
  }
  FsmArgs f{n, 0, 7, st.data(), tg.data(), ok.data(), t0.data(), t1.data()};
  fsm_host(f);
  // breach windows with a tiny ring capacity (wrap-around)
  const int P = 33, W = 7;
  std::vector<int64_t> now(P), ts(P * W), tot(P), tat(P);
  std::vector<uint8_t> ar(P), nc(P), called(P * W), trip(P), sev(P), evt(P);
  std::vector<int32_t> head(P), cnt(P), hits(P);
  std::vector<double> rate(P);
  for (int step = 0; step < 50; ++step) {
    for (int p = 0; p < P; ++p) {
      now[p] = step * 1'000'000LL * rnd(1, 3);
      ar[p] = static_cast<uint8_t>(rnd(1, 3));
      nc[p] = static_cast<uint8_t>(rnd(0, 3));
    }
    BreachArgs b{P, W, 60'000'000, 30'000'000, nullptr, nullptr, now.data(), ar.data(), nc.data(), ts.data(),
                 called.data(), head.data(), cnt.data(), tot.data(), trip.data(), tat.data(), nullptr, sev.data(),
                 rate.data(), hits.data(), evt.data(), nullptr};
    breach_host(b);
  }
  for (int p = 0; p < P; ++p) CHECK(cnt[p] <= W && tot[p] == 50);
  // ledger / drift / attribution
  std::vector<int32_t> loff{0};
  std::vector<uint8_t> lt;
  std::vector<double> lsev;
  for (int a = 0; a < 40; ++a) {
    for (int e = rnd(0, 12); e > 0; --e) {
      lt.push_back(static_cast<uint8_t>(rnd(0, 8)));
      lsev.push_back(rndf());
    }
    loff.push_back(static_cast<int32_t>(lt.size()));
  }
  std::vector<double> raw(40), risk(40), favg(40);
  std::vector<uint8_t> rec(40);
  std::vector<int32_t> sc(40), qc(40), cc(40);
  LedgerArgs la{40, loff.data(), lt.data(), lsev.data(), raw.data(), risk.data(), rec.data(), sc.data(), qc.data(),
                cc.data(), favg.data()};
  ledger_host(la);
  for (double x : risk) CHECK(x >= 0.0 && x <= 1.0);
}

// ----------------------------------------------------------------- session
static void test_session() {
  const int G = 5, A = 9, per = 40;
  std::vector<int32_t> off(G + 1), path(G * per), agent(G * per), col(G * per);
  std::vector<uint8_t> op(G * per), ok(G * per);
  for (int g = 0; g <= G; ++g) off[g] = g * per;
  for (int q = 0; q < G * per; ++q) {
    const int g = q / per;
    op[q] = rnd(0, 1);
    path[q] = g * 3 + rnd(0, 2);
    col[q] = rnd(0, A - 1);
    agent[q] = g * A + col[q];
  }
  std::vector<uint32_t> pc(G * 3 * A), ac(G * A * A);
  VClockArgs v{G, A, 1, off.data(), op.data(), path.data(), agent.data(), col.data(), pc.data(), ac.data(),
               ok.data()};
  vclock_host(v);
  std::vector<int32_t> roff{0, 2, 2, 5}, la{1, 2, 3, 4, 5}, rr{0, 1, 2, 2}, ra{1, 9, 3, 7}, conf(4);
  std::vector<uint8_t> li{0, 1, 0, 0, 2}, ri{0, 1, 0, 2};
  LockArgs l{4, roff.data(), la.data(), li.data(), rr.data(), ra.data(), ri.data(), conf.data()};
  locks_host(l);
  CHECK(conf[0] == 1 && conf[1] == 0 && conf[2] == 1 && conf[3] == 3);
}

// Strings of the batched pipelines' pool (16-byte aligned, padded).
struct Pool {
  std::vector<uint8_t> bytes;
  std::vector<int64_t> off;
  std::vector<int32_t> len;
  int32_t add(const std::string& s) {
    off.push_back(static_cast<int64_t>(bytes.size()));
    len.push_back(static_cast<int32_t>(s.size()));
    bytes.insert(bytes.end(), s.begin(), s.end());
    while (bytes.size() % 16) bytes.push_back(0);
    return static_cast<int32_t>(len.size() - 1);
  }
};

// ------------------------------------------------------------------ store
// The device state store's command set (ahv/store.h) through StoreCore's host
// twin — the same store_exec body the resident gfx950 worker runs — driven by
// random programs that touch every OP_*: session lifecycle, captures with the
// chain re-derived on the host, Merkle / verify / read commands, liability
// edges and slashing, sagas, row reclaim and reuse (OP_FREE_ROWS), table growth
// (rebind), arena growth, reserve_deltas + the template pipeline kernel's host
// twin, and malformed row arguments that must come back as errors.  A shadow
// model of every live row checks the statuses and the read-backs.
namespace sto = ahv::store;
using ahv::host::ColumnPtrs;
using ahv::host::Placed;
using ahv::host::StoreCore;
using sto::bitsd;
using sto::dbits;

// Host-memory columns (the tensors agent_hypervisor_amd/models/store.py
// allocates) with the same fill rules: free markers are all-ones bytes (-1 /
// 255), everything else zero.  Growth keeps every old row in place.
struct HostCols {
  sto::Caps cap{};
  std::map<std::string, std::vector<uint8_t>> col;
  static bool ones(const std::string& n) {
    static const char* k[] = {"v_head", "v_tail", "s_dlast", "d_prev", "e_next", "d_sess",
                              "e_vsess", "t_saga", "d_hole", "s_state", "g_state", "t_state"};
    for (const char* x : k)
      if (n == x) return true;
    return false;
  }
  static int64_t extent(const sto::Caps& c, const std::string& e) {
    if (e == "S") return c.S;
    if (e == "S4") return 4 * c.S;
    if (e == "S8") return 8 * c.S;
    if (e == "SP") return c.S * c.P;
    if (e == "D") return c.D;
    if (e == "D8") return 8 * c.D;
    if (e == "E") return c.E;
    if (e == "V") return c.V;
    if (e == "G") return c.G;
    if (e == "T") return c.T;
    if (e == "SCR") return c.X;
    throw std::logic_error("unknown extent " + e);
  }
  void grow_col(const std::string& n, size_t es, int64_t ext, bool sp, const sto::Caps& c) {
    std::vector<uint8_t> v(static_cast<size_t>(ext) * es, ones(n) ? 0xFF : 0);
    auto it = col.find(n);
    if (it != col.end()) {
      if (sp) {  // participant-major [P][S] (store.h prow): each participant plane keeps its rows
        for (int64_t k = 0; k < c.P; ++k)
          std::memcpy(v.data() + static_cast<size_t>(k * c.S) * es, it->second.data() + static_cast<size_t>(k * cap.S) * es,
                      static_cast<size_t>(cap.S) * es);
      } else {
        std::memcpy(v.data(), it->second.data(), std::min(v.size(), it->second.size()));
      }
    }
    col[n] = std::move(v);
  }
  void resize(const sto::Caps& c) {
#define AHV_COL(name, type, ext) grow_col(#name, sizeof(type), extent(c, #ext), std::string(#ext) == "SP", c);
    AHV_STORE_COLUMNS(AHV_COL)
#undef AHV_COL
    cap = c;
  }
  ColumnPtrs ptrs() {
    ColumnPtrs p;
    for (auto& kv : col) p[kv.first] = reinterpret_cast<uintptr_t>(kv.second.data());
    return p;
  }
};

static std::vector<uint32_t> merkle_of(const std::vector<uint32_t>& leaves) {
  const int32_t n = static_cast<int32_t>(leaves.size() / 8);
  std::vector<uint32_t> scratch(std::max<size_t>(leaves.size(), 8)), root(8, 0);
  int32_t offs[2] = {0, n};
  MerkleArgs m{};
  m.chains = 1;
  m.offsets = offs;
  m.leaves = leaves.data();
  m.scratch = scratch.data();
  m.root = root.data();
  merkle_host(m);
  return root;
}

static std::string render_record(const std::string& sid, int turn, int64_t ts, size_t pad, size_t* at) {
  std::string s = "{\"agent_did\": \"did:mesh:fuzz\", \"changes\": [{\"path\": \"/f" + std::to_string(turn) +
                  std::string(pad, 'p') + "\"}], \"delta_id\": \"delta:" + std::to_string(turn) +
                  "\", \"parent_hash\": ";
  *at = s.size();
  s += "null, \"session_id\": \"" + sid + "\", \"timestamp\": " + std::to_string(ts) +
       ", \"turn_id\": " + std::to_string(turn) + "}";
  return s;
}

static void put_hex(uint8_t* dst, const uint32_t* d) {
  const std::string h = hex(d);
  dst[0] = '"';
  std::memcpy(dst + 1, h.data(), 64);
  dst[65] = '"';
}

struct FzSess {
  int64_t row;
  uint64_t stamp;
  uint8_t state;
  int32_t maxpart;
  double minsig;
  int32_t pactive = 0;
  std::vector<int32_t> agents;
  std::vector<uint8_t> active;
  std::vector<int32_t> drows;
  std::string sid;
};
struct FzSaga {
  int64_t row;
  uint8_t state;
  std::vector<int32_t> steps;
  std::vector<uint8_t> sstate;
};
struct FzVs {
  int32_t row;
  std::vector<int32_t> edges;
};

class StoreFuzz {
 public:
  explicit StoreFuzz(uint64_t seed) : rg(seed) {
    sto::Caps c{16, 4, 48, 16, 4, 8, 16, 1 << 16, 4096};
    cols.resize(c);
    core.reset(new StoreCore(-1, cols.ptrs(), c, 8, 1 << 18, 1 << 18, 0, 0));
    pool_creator = pool.add("did:mesh:admin");
    for (int a = 0; a < kAgents; ++a) {
      agent_pool.push_back(pool.add("did:mesh:fuzz-agent-" + std::to_string(a) + std::string(a % 5 * 7, 'x')));
      agent_sigma.push_back(0.3 + 0.7 * rndf());
      agent_id.push_back(a);
    }
    for (int d = 0; d < 8 * 4; ++d)
      changes.push_back(ChangeIds{pool.add("/p" + std::to_string(d)), pool.add(d % 3 ? "add" : "modify"),
                                  pool.add("h" + std::to_string(d)), d % 4 ? -1 : pool.add("prev")});
  }

  void run(int steps) {
    for (int i = 0; i < steps; ++i) {
      now += rnd(1, 50);
      step();
      if (i % 97 == 0) check_all();
    }
    check_all();
    // every opcode the store defines was issued at least once
    const uint32_t all[] = {sto::OP_NOP, sto::OP_STOP, sto::OP_FLUSH, sto::OP_ACQUIRE, sto::OP_FREE_ROWS,
                            sto::OP_SESS_CREATE, sto::OP_SESS_JOIN, sto::OP_SESS_LEAVE, sto::OP_SESS_ACTIVATE,
                            sto::OP_SESS_TERMINATE, sto::OP_SESS_ARCHIVE, sto::OP_SESS_UPDATE_RING,
                            sto::OP_SESS_SET_MODE, sto::OP_SESS_READ, sto::OP_SESS_SET_SIGMA, sto::OP_SESS_CLOSE,
                            sto::OP_SESS_HANDSHAKE, sto::OP_SESS_READ_MANY, sto::OP_DELTA_CAPTURE,
                            sto::OP_DELTA_MERKLE, sto::OP_DELTA_VERIFY, sto::OP_DELTA_READ, sto::OP_VOUCH,
                            sto::OP_SIGMA_EFF, sto::OP_EXPOSURE, sto::OP_RELEASE_BOND, sto::OP_RELEASE_SESSION,
                            sto::OP_VOUCH_LIST, sto::OP_EDGE_READ, sto::OP_SLASH, sto::OP_V_RETIRE,
                            sto::OP_SAGA_CREATE, sto::OP_STEP_ADD, sto::OP_STEP_TRANSITION, sto::OP_STEP_SET,
                            sto::OP_SAGA_TRANSITION, sto::OP_SAGA_READ, sto::OP_SAGA_PLAN, sto::OP_STEP_READ};
    for (uint32_t op : all) {
      if (!seen[op]) std::fprintf(stderr, "store fuzz: opcode %u never issued\n", op);
      CHECK(seen[op] > 0);
    }
    CHECK(grows_S > 0 && grows_B > 0 && reused > 0 && template_sessions > 0);
  }

  int grows_S = 0, grows_D = 0, grows_E = 0, grows_B = 0, reused = 0, template_sessions = 0;

 private:
  static constexpr int kAgents = 12;
  std::mt19937_64 rg;
  HostCols cols;
  std::unique_ptr<StoreCore> core;
  Pool pool;
  int32_t pool_creator;
  std::vector<int32_t> agent_pool, agent_id;
  std::vector<double> agent_sigma;
  std::vector<ChangeIds> changes;
  std::vector<FzSess> sess;
  std::vector<FzSaga> sagas;
  std::vector<FzVs> vss;
  std::vector<int64_t> freed_s;  // session rows released (a later create on one is a reuse)
  int64_t now = 1'767'225'600'000'000LL;
  uint64_t id_base = 0;
  uint64_t seen[128] = {};

  int rnd(int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rg); }
  double rndf() { return std::uniform_real_distribution<double>(0.0, 1.0)(rg); }
  template <class T>
  T& pick(std::vector<T>& v) { return v[static_cast<size_t>(rnd(0, static_cast<int>(v.size()) - 1))]; }
  const sto::Tables& T() const { return core->tables(); }

  const uint64_t* call(uint32_t op, std::vector<uint64_t> a, const void* inl = nullptr, size_t nb = 0) {
    ++seen[op & 127];
    return core->wait(core->post_raw(op, a.data(), a.size(), static_cast<const uint8_t*>(inl), nb));
  }
  // An index list: inline when it fits the slot, else staged (returns the staging offset).
  const uint64_t* call_list(uint32_t op, std::vector<uint64_t> a, size_t off_pos, const std::vector<int32_t>& idx) {
    if (idx.size() <= static_cast<size_t>(2 * sto::kInlineWords)) return call(op, a, idx.data(), 4 * idx.size());
    a[off_pos] = static_cast<uint64_t>(core->stage_raw(reinterpret_cast<const uint8_t*>(idx.data()), 4 * idx.size()));
    return call(op, a);
  }

  void grow(char k) {
    sto::Caps c = cols.cap;
    c.B = core->payload_cap();
    if (k == 'S') c.S *= 2, ++grows_S;
    if (k == 'D') c.D *= 2, ++grows_D;
    if (k == 'E') c.E *= 2, ++grows_E;
    if (k == 'V') c.V *= 2;
    if (k == 'G') c.G *= 2;
    if (k == 'T') c.T *= 2;
    core->quiesce();
    cols.resize(c);
    core->rebind(cols.ptrs(), c);
  }
  int64_t row(uint64_t kind, char k) {
    int64_t r = core->alloc_row(kind);
    if (r < 0) {
      grow(k);
      r = core->alloc_row(kind);
    }
    CHECK(r >= 0);
    return r;
  }
  int64_t bad_index(int64_t cap) { return rnd(0, 1) ? -rnd(1, 3) : cap + rnd(0, 3); }

  // ------------------------------------------------------------- model checks
  // Re-derive a session's chain on the host: row links, the record bytes with the
  // parent digest spliced into the hole, SHA-256 against d_hash, and the head.
  std::vector<uint32_t> chain(const FzSess& f, bool* ok) {
    const sto::Tables& t = T();
    std::vector<uint32_t> out;
    *ok = true;
    const uint32_t* prev = nullptr;
    for (size_t k = 0; k < f.drows.size(); ++k) {
      const int32_t d = f.drows[k];
      if (t.d_sess[d] != f.row || t.d_turn[d] != static_cast<int32_t>(k + 1) ||
          t.d_prev[d] != (k ? f.drows[k - 1] : -1)) {
        std::fprintf(stderr, "chain: session row %lld (%s) delta %zu row %d: sess %d turn %d prev %d\n",
                     static_cast<long long>(f.row), f.sid.c_str(), k, d, t.d_sess[d], t.d_turn[d], t.d_prev[d]);
        *ok = false;
        return out;
      }
      std::vector<uint8_t> b(static_cast<size_t>(t.d_len[d]));
      core->payload_read(t.d_off[d], t.d_len[d], b.data());
      const int32_t hole = t.d_hole[d];
      if ((k > 0) != (hole >= 0) || (hole >= 0 && static_cast<size_t>(hole) + 66 > b.size())) {
        *ok = false;
        return out;
      }
      if (hole >= 0) put_hex(b.data() + hole, prev);
      uint32_t h[8];
      sto::sha256_mem(b.data(), b.size(), h);
      if (std::memcmp(h, t.d_hash + 8 * static_cast<int64_t>(d), 32) != 0) {
        std::fprintf(stderr, "chain: session row %lld (%s) delta %zu: digest mismatch (hole %d, len %d)\n",
                     static_cast<long long>(f.row), f.sid.c_str(), k, hole, t.d_len[d]);
        *ok = false;
        return out;
      }
      out.insert(out.end(), h, h + 8);
      prev = t.d_hash + 8 * static_cast<int64_t>(d);
    }
    if (prev && std::memcmp(prev, t.s_head + 8 * f.row, 32) != 0) {
      std::fprintf(stderr, "chain: session row %lld (%s): head != last digest\n", static_cast<long long>(f.row),
                   f.sid.c_str());
      *ok = false;
    }
    return out;
  }

  void check_all() {
    const sto::Tables& t = T();
    for (const FzSess& f : sess) {
      bool ok;
      chain(f, &ok);
      CHECK(ok);
      CHECK(t.s_state[f.row] == f.state);
      CHECK(t.s_dcount[f.row] == static_cast<int32_t>(f.drows.size()));
      CHECK(t.s_pcount[f.row] == static_cast<int32_t>(f.agents.size()));
      CHECK(t.s_pactive[f.row] == f.pactive);
      CHECK(sto::row_stamp(t, f.row) == f.stamp);
    }
    for (const FzSaga& g : sagas) {
      CHECK(t.g_state[g.row] == g.state && t.g_nsteps[g.row] == static_cast<int32_t>(g.steps.size()));
      for (size_t k = 0; k < g.steps.size(); ++k)
        CHECK(t.t_state[g.steps[k]] == g.sstate[k] && t.t_saga[g.steps[k]] == g.row);
    }
    for (const FzVs& v : vss) {
      int32_t e = t.v_head[v.row];
      for (int32_t x : v.edges) {
        CHECK(e == x);
        if (e != x) break;
        CHECK(t.e_vsess[e] == v.row);
        e = t.e_next[e];
      }
      CHECK(e == -1 || v.edges.empty());
    }
  }

  // ------------------------------------------------------------- sessions
  void create() {
    const int64_t r = row(sto::RK_S, 'S');
    if (std::find(freed_s.begin(), freed_s.end(), r) != freed_s.end()) ++reused;
    const uint64_t hi = rg() & 0xFFFFFFFFFFFF0FFFull, lo = (rg() | 1ull) & 0x3FFFFFFFFFFFFFFFull;
    const bool bare = rnd(0, 3) == 0;
    FzSess f{r, lo, static_cast<uint8_t>(bare ? SS_CREATED : SS_HANDSHAKING), rnd(1, 5), 0.2 * rndf()};
    f.sid = "session:" + std::to_string(r) + "-" + std::to_string(lo % 1000);
    const uint64_t* q = call(sto::OP_SESS_CREATE, {static_cast<uint64_t>(r), static_cast<uint64_t>(rnd(0, kAgents)),
                                                   static_cast<uint64_t>(now), static_cast<uint64_t>(rnd(0, 2)),
                                                   static_cast<uint64_t>(f.maxpart), dbits(f.minsig), 1, hi, lo,
                                                   bare ? 1ull : 0ull});
    CHECK(q[1] == sto::ST_OK);
    sess.push_back(f);
  }
  void create_on_live() {  // a create never overwrites a live row
    if (sess.empty()) return;
    FzSess& f = pick(sess);
    const uint64_t* q = call(sto::OP_SESS_CREATE, {static_cast<uint64_t>(f.row), 0, 0, 0, 1, 0, 1, 7, 9, 0});
    CHECK(q[1] == sto::ST_BAD_STATE && q[2] == f.state);
  }
  uint64_t stamp_arg(const FzSess& f, bool* wrong) {
    const int k = rnd(0, 9);
    *wrong = k == 0;
    return k == 0 ? (f.stamp ^ 0x10) : (k < 5 ? f.stamp : 0);
  }
  void join() {
    if (sess.empty()) return;
    FzSess& f = pick(sess);
    const int32_t agent = rnd(0, kAgents - 1);
    const double sraw = rndf(), seff = rnd(0, 4) ? 0.3 + 0.7 * rndf() : rndf();
    const uint64_t flags = static_cast<uint64_t>(rnd(0, 3)), ringv = static_cast<uint64_t>(rnd(0, 3));
    bool wrong;
    const uint64_t stamp = stamp_arg(f, &wrong);
    const uint64_t* q = call(sto::OP_SESS_JOIN, {static_cast<uint64_t>(f.row), static_cast<uint64_t>(agent),
                                                 dbits(sraw), dbits(seff), flags, ringv, static_cast<uint64_t>(now),
                                                 stamp});
    uint64_t want;
    if (wrong) {
      want = sto::JOIN_NOT_MINE;
    } else {
      uint8_t ring = (flags & 2u) ? static_cast<uint8_t>(ringv) : ring_from_sigma(seff, false);
      if (!(flags & 2u) && !(flags & 1u)) ring = RING3;
      const bool dup = std::find(f.agents.begin(), f.agents.end(), agent) != f.agents.end();
      want = join_check(f.state, dup, f.pactive, f.maxpart, seff, f.minsig, ring);
      if (want == JOIN_OK && static_cast<int64_t>(f.agents.size()) >= T().cap.P) want = sto::JOIN_ROWS;
    }
    CHECK(q[1] == want);
    if (q[1] == JOIN_OK) {
      f.agents.push_back(agent);
      f.active.push_back(1);
      f.pactive += 1;
    }
  }
  void leave() {
    if (sess.empty()) return;
    FzSess& f = pick(sess);
    const int32_t agent = rnd(0, kAgents - 1);
    const uint64_t* q = call(sto::OP_SESS_LEAVE, {static_cast<uint64_t>(f.row), static_cast<uint64_t>(agent)});
    auto it = std::find(f.agents.begin(), f.agents.end(), agent);
    CHECK(q[1] == (it == f.agents.end() ? sto::ST_NOT_FOUND : sto::ST_OK));
    if (it != f.agents.end()) {
      const size_t k = static_cast<size_t>(it - f.agents.begin());
      if (f.active[k]) f.pactive -= 1;
      f.active[k] = 0;
    }
  }
  void tweak() {
    if (sess.empty()) return;
    FzSess& f = pick(sess);
    const int32_t agent = rnd(0, kAgents - 1);
    const bool found = std::find(f.agents.begin(), f.agents.end(), agent) != f.agents.end();
    const uint64_t s = static_cast<uint64_t>(f.row), a = static_cast<uint64_t>(agent);
    const uint64_t* q;
    switch (rnd(0, 2)) {
      case 0:
        q = call(sto::OP_SESS_UPDATE_RING, {s, a, static_cast<uint64_t>(rnd(0, 3))});
        CHECK(q[1] == (found ? sto::ST_OK : sto::ST_NOT_FOUND));
        break;
      case 1:
        q = call(sto::OP_SESS_SET_SIGMA, {s, a, dbits(rndf()), static_cast<uint64_t>(rnd(0, 1)), 2});
        CHECK(q[1] == (found ? sto::ST_OK : sto::ST_NOT_FOUND));
        break;
      default:
        q = call(sto::OP_SESS_SET_MODE, {s, static_cast<uint64_t>(rnd(0, 2))});
        CHECK(q[1] == sto::ST_OK);
    }
  }
  void lifecycle() {
    if (sess.empty()) return;
    FzSess& f = pick(sess);
    const uint64_t s = static_cast<uint64_t>(f.row);
    switch (rnd(0, 3)) {
      case 0: {
        const uint64_t* q = call(sto::OP_SESS_HANDSHAKE, {s});
        CHECK(q[1] == (f.state == SS_CREATED ? sto::ST_OK : sto::ST_BAD_STATE));
        if (q[1] == sto::ST_OK) f.state = SS_HANDSHAKING;
        break;
      }
      case 1: {
        bool wrong;
        const uint64_t* q = call(sto::OP_SESS_ACTIVATE, {s, stamp_arg(f, &wrong)});
        const uint64_t want = wrong ? sto::ACT_NOT_MINE
                                    : (f.state != SS_HANDSHAKING ? sto::ST_BAD_STATE : (f.agents.empty() ? 3u : sto::ST_OK));
        CHECK(q[1] == want);
        if (q[1] == sto::ST_OK) f.state = SS_ACTIVE;
        break;
      }
      case 2: {
        const uint64_t* q = call(sto::OP_SESS_TERMINATE, {s, static_cast<uint64_t>(now)});
        const bool ok = (session_op_allowed_from(OP_TERMINATE) >> f.state) & 1u;
        CHECK(q[1] == (ok ? sto::ST_OK : sto::ST_BAD_STATE));
        if (ok) f.state = SS_TERMINATING;
        break;
      }
      default: {
        const uint64_t* q = call(sto::OP_SESS_ARCHIVE, {s});
        CHECK(q[1] == (f.state == SS_TERMINATING ? sto::ST_OK : sto::ST_BAD_STATE));
        if (q[1] == sto::ST_OK) f.state = SS_ARCHIVED;
      }
    }
  }
  void bad_session_args() {
    const uint64_t s = static_cast<uint64_t>(bad_index(T().cap.S));
    const uint32_t ops[] = {sto::OP_SESS_JOIN, sto::OP_SESS_LEAVE, sto::OP_SESS_ACTIVATE, sto::OP_SESS_TERMINATE,
                            sto::OP_SESS_ARCHIVE, sto::OP_SESS_UPDATE_RING, sto::OP_SESS_SET_MODE,
                            sto::OP_SESS_SET_SIGMA, sto::OP_SESS_HANDSHAKE, sto::OP_SESS_READ, sto::OP_SESS_CREATE};
    const uint64_t* q = call(ops[rnd(0, 10)], {s, 1, 2, 3, 0, 0, 0, 0, 0, 0});
    CHECK(q[1] == sto::ST_BAD_ARG);
    // an unassigned code in each range
    const uint32_t unk[] = {5, 9, 23, 29, 34, 39, 49, 59, 68, 79, 80, 127};
    const uint32_t op = unk[rnd(0, 11)];
    const uint64_t live = sess.empty() ? 0 : static_cast<uint64_t>(pick(sess).row);
    q = call(op, {live, 0, 0, 0});
    if (sess.empty() && op >= 10 && op < 30) CHECK(q[1] == sto::ST_BAD_ARG || q[1] == sto::ST_BAD_OP);
    else CHECK(q[1] == sto::ST_BAD_OP);
  }

  // ------------------------------------------------------------- audit
  void capture() {
    if (sess.empty()) return;
    FzSess& f = pick(sess);
    if (f.drows.size() >= 24) return;
    const int turn = static_cast<int>(f.drows.size()) + 1;
    size_t at;
    const size_t pad = rnd(0, 60) == 0 ? 17000 : static_cast<size_t>(rnd(0, 200));
    const std::string rec = render_record(f.sid, turn, now, pad, &at);
    for (int tries = 0; tries < 4; ++tries) {
      const Placed p = core->capture_rendered(f.row, turn, now, rec, at);
      if (p.didx == -3) {
        core->grow_payload(std::max<int64_t>(2 * core->payload_cap(), core->payload_cap() + 2 * p.len));
        ++grows_B;
        continue;
      }
      if (p.didx == -2) {
        if (core->reclaim_pool(sto::RK_D) == 0) grow('D');
        continue;
      }
      CHECK(core->wait(static_cast<uint64_t>(p.seq))[1] == sto::ST_OK);
      f.drows.push_back(static_cast<int32_t>(p.didx));
      return;
    }
    CHECK(false);
  }
  void bad_capture() {  // always refused: wrong turn or out-of-range rows / bytes
    const sto::Tables& t = T();
    int64_t s = rnd(0, 2) ? (sess.empty() ? 0 : pick(sess).row) : bad_index(t.cap.S);
    const int32_t dc = (s >= 0 && s < t.cap.S) ? t.s_dcount[s] : 0;
    const uint64_t* q = call(sto::OP_DELTA_CAPTURE,
                             {static_cast<uint64_t>(s), static_cast<uint64_t>(rnd(0, 1) ? bad_index(t.cap.D) : 0),
                              static_cast<uint64_t>(dc + 2 + rnd(0, 3)), static_cast<uint64_t>(now),
                              static_cast<uint64_t>(rnd(0, 1) ? t.cap.B : 0), 100, ~0ull});
    CHECK(q[1] == sto::ST_BAD_ARG);
  }
  void merkle() {
    if (sess.empty()) return;
    FzSess& f = pick(sess);
    bool ok;
    const std::vector<uint32_t> lv = chain(f, &ok);
    CHECK(ok);
    std::vector<int32_t> idx = f.drows;
    const int mode = rnd(0, 7);
    if (mode == 0 && !idx.empty()) std::swap(idx.front(), idx.back());  // out of order
    uint64_t n = idx.size();
    if (mode == 1) n += 1;  // count mismatch
    if (mode == 1) idx.push_back(0);
    const uint64_t* q = call_list(sto::OP_DELTA_MERKLE, {static_cast<uint64_t>(f.row), n, 0}, 2, idx);
    const bool bad = mode == 1 || (mode == 0 && idx.size() > 1);
    CHECK(q[1] == (bad ? sto::ST_BAD_ARG : sto::ST_OK));
    if (!bad) {
      CHECK(q[2] == (n > 0 ? 1u : 0u));
      if (n > 0) {
        const std::vector<uint32_t> root = merkle_of(lv);
        for (int k = 0; k < 8; ++k) CHECK(q[3 + k] == root[k]);
      }
    }
  }
  void verify() {
    if (sess.empty()) return;
    FzSess& f = pick(sess);
    if (f.drows.empty()) return;
    const sto::Tables& t = T();
    const size_t n = f.drows.size();
    std::vector<std::vector<uint8_t>> recs(n);
    size_t total = 0;
    const uint32_t* prev = nullptr;
    for (size_t k = 0; k < n; ++k) {
      const int32_t d = f.drows[k];
      recs[k].resize(static_cast<size_t>(t.d_len[d]));
      core->payload_read(t.d_off[d], t.d_len[d], recs[k].data());
      if (t.d_hole[d] >= 0) put_hex(recs[k].data() + t.d_hole[d], prev);
      prev = t.d_hash + 8 * static_cast<int64_t>(d);
      total += recs[k].size() + 64;
    }
    if (total + n * 88 > static_cast<size_t>(core->staging_cap()) / 2) return;
    const int tamper = rnd(0, 2) == 0 ? rnd(0, static_cast<int>(n) - 1) : -1;
    if (tamper >= 0) recs[static_cast<size_t>(tamper)][10] ^= 1;
    std::vector<uint64_t> table(11 * n);
    for (size_t k = 0; k < n; ++k) {
      const int32_t d = f.drows[k];
      table[11 * k + 0] = static_cast<uint64_t>(core->stage_raw(recs[k].data(), recs[k].size()));
      table[11 * k + 1] = recs[k].size();
      table[11 * k + 2] = static_cast<uint64_t>(d);
      std::memcpy(&table[11 * k + 3], t.d_hash + 8 * static_cast<int64_t>(d), 32);
      if (k == 0) std::memset(&table[11 * k + 7], 0xFF, 32);
      else std::memcpy(&table[11 * k + 7], t.d_hash + 8 * static_cast<int64_t>(f.drows[k - 1]), 32);
    }
    const uint64_t toff = static_cast<uint64_t>(core->stage_raw(reinterpret_cast<const uint8_t*>(table.data()),
                                                                8 * table.size()));
    const bool parity = rnd(0, 1);
    const uint64_t* q = call(sto::OP_DELTA_VERIFY, {static_cast<uint64_t>(f.row), n, toff, parity ? 1u : 0u, 0});
    CHECK(q[1] == sto::ST_OK);
    int64_t want_bad = -1;
    if (tamper >= 0) want_bad = parity ? (static_cast<size_t>(tamper) + 1 < n ? tamper + 1 : -1) : tamper;
    CHECK(q[2] == (want_bad < 0 ? 1u : 0u));
    if (want_bad >= 0) CHECK(static_cast<int64_t>(q[3]) == want_bad);
  }
  void delta_read() {
    if (sess.empty()) return;
    FzSess& f = pick(sess);
    std::vector<int32_t> idx = f.drows;
    const bool bad = rnd(0, 5) == 0;
    if (bad) idx.push_back(static_cast<int32_t>(bad_index(T().cap.D)));
    const uint64_t* q = call_list(sto::OP_DELTA_READ, {idx.size(), 0, 0}, 1, idx);
    CHECK(q[1] == (bad ? sto::ST_BAD_ARG : sto::ST_OK));
    if (!bad) {
      const uint64_t* b = reinterpret_cast<const uint64_t*>(core->bulk_ptr(0, 96 * static_cast<int64_t>(idx.size())));
      for (size_t k = 0; k < idx.size(); ++k) {
        CHECK(static_cast<int64_t>(b[12 * k]) == static_cast<int64_t>(k + 1));
        CHECK(static_cast<int64_t>(b[12 * k + 3]) == f.row);
      }
    }
  }
  void reads() {
    if (sess.empty()) return;
    if (rnd(0, 1)) {
      FzSess& f = pick(sess);
      const uint64_t* q = call(sto::OP_SESS_READ, {static_cast<uint64_t>(f.row), 0});
      CHECK(q[1] == sto::ST_OK && q[2] == f.state && q[4] == f.agents.size() &&
            q[5] == static_cast<uint64_t>(f.pactive) && q[8] == f.drows.size());
      const uint64_t* b = reinterpret_cast<const uint64_t*>(core->bulk_ptr(0, 40 * T().cap.P));
      for (size_t k = 0; k < f.agents.size(); ++k) CHECK(static_cast<int32_t>(b[5 * k]) == f.agents[k]);
      return;
    }
    std::vector<int32_t> idx;
    for (const FzSess& f : sess) idx.push_back(static_cast<int32_t>(f.row));
    const bool parts = rnd(0, 1);
    const uint64_t* q = call_list(sto::OP_SESS_READ_MANY, {idx.size(), 0, 0, parts ? 1u : 0u}, 1, idx);
    CHECK(q[1] == sto::ST_OK);
    const int64_t words = static_cast<int64_t>(idx.size()) * (sto::kHdrWords + (parts ? 5 * T().cap.P : 0));
    const uint64_t* b = reinterpret_cast<const uint64_t*>(core->bulk_ptr(0, 8 * words));
    for (size_t i = 0; i < sess.size(); ++i) {
      const uint64_t* h = b + sto::kHdrWords * i;
      CHECK((h[0] & 0xFF) == sess[i].state);
      CHECK((h[1] & 0xFFFFFFFFu) == sess[i].agents.size());
      CHECK((h[4] & 0xFFFFFFFFu) == sess[i].drows.size());
      CHECK(h[11] == sess[i].stamp);
    }
  }
  void close() {
    if (sess.empty()) return;
    FzSess& f = pick(sess);
    bool ok;
    const std::vector<uint32_t> lv = chain(f, &ok);
    const int64_t v = vss.empty() || rnd(0, 1) ? -1 : pick(vss).row;
    const uint64_t* q = call_list(sto::OP_SESS_CLOSE,
                                  {static_cast<uint64_t>(f.row), f.drows.size(), 0, static_cast<uint64_t>(now),
                                   static_cast<uint64_t>(v), static_cast<uint64_t>(now - 100), 1},
                                  2, f.drows);
    const bool allowed = (session_op_allowed_from(OP_TERMINATE) >> f.state) & 1u;
    CHECK(q[1] == (allowed ? sto::ST_OK : sto::ST_BAD_STATE));
    if (!allowed) return;
    f.state = SS_ARCHIVED;
    if (!f.drows.empty()) {
      const std::vector<uint32_t> root = merkle_of(lv);
      CHECK(std::memcmp(root.data(), T().s_root + 8 * f.row, 32) == 0);
    }
  }
  void release_session() {
    if (sess.empty()) return;
    const size_t i = static_cast<size_t>(rnd(0, static_cast<int>(sess.size()) - 1));
    const FzSess f = sess[i];
    sess.erase(sess.begin() + static_cast<std::ptrdiff_t>(i));
    if (!f.drows.empty()) core->release_rows_raw(sto::RK_D, f.drows.data(), static_cast<int64_t>(f.drows.size()));
    if (rnd(0, 2) == 0) core->reclaim_pool(sto::RK_D);
    core->release_row(sto::RK_S, f.row);
    freed_s.push_back(f.row);
    if (rnd(0, 3) == 0) core->reclaim_pool(sto::RK_S);
  }

  // ------------------------------------------------------------- liability
  void vouch() {
    if (vss.empty() || rnd(0, 6) == 0) {
      vss.push_back(FzVs{static_cast<int32_t>(row(sto::RK_V, 'V')), {}});
      return;
    }
    FzVs& v = pick(vss);
    const int64_t e = row(sto::RK_E, 'E');
    const int32_t vr = rnd(0, 7), ve = rnd(0, 7);
    const double sigma = 0.4 + 0.6 * rndf();
    const uint64_t pct = rnd(0, 1) ? dbits(std::nan("")) : dbits(rndf());
    const int64_t expiry = rnd(0, 3) ? -1 : now + rnd(-20, 200);
    const uint64_t* q = call(sto::OP_VOUCH, {static_cast<uint64_t>(v.row), static_cast<uint64_t>(vr),
                                             static_cast<uint64_t>(ve), dbits(sigma), pct,
                                             static_cast<uint64_t>(expiry), static_cast<uint64_t>(now), dbits(0.8),
                                             static_cast<uint64_t>(rnd(0, 1)), static_cast<uint64_t>(e)});
    if (vr == ve) CHECK(q[1] == sto::V_SELF);
    else if (sigma < 0.5) CHECK(q[1] == sto::V_LOW_SIGMA);
    if (q[1] == sto::V_OK) {
      v.edges.push_back(static_cast<int32_t>(e));
    } else {
      CHECK(q[1] == sto::V_SELF || q[1] == sto::V_LOW_SIGMA || q[1] == sto::V_CYCLE || q[1] == sto::V_EXPOSURE);
      core->return_row(sto::RK_E, e);
    }
    if (!v.edges.empty() && rnd(0, 3) == 0) {  // an edge row in use is refused
      q = call(sto::OP_VOUCH, {static_cast<uint64_t>(v.row), 1, 2, dbits(0.9), pct, ~0ull,
                               static_cast<uint64_t>(now), dbits(0.8), 0, static_cast<uint64_t>(pick(v.edges))});
      CHECK(q[1] == sto::ST_BAD_STATE);
    }
    q = call(sto::OP_VOUCH, {static_cast<uint64_t>(bad_index(T().cap.V)), 1, 2, dbits(0.9), pct, ~0ull, 0,
                             dbits(0.8), 0, 0});
    CHECK(q[1] == sto::ST_BAD_ARG);
  }
  void liability_reads() {
    if (vss.empty()) return;
    FzVs& v = pick(vss);
    const uint64_t vr = static_cast<uint64_t>(v.row), t = static_cast<uint64_t>(now);
    const uint64_t* q = call(sto::OP_SIGMA_EFF, {vr, static_cast<uint64_t>(rnd(0, 7)), dbits(rndf()), dbits(rndf()), t});
    CHECK(q[1] == sto::ST_OK && bitsd(q[2]) <= 1.0);
    q = call(sto::OP_EXPOSURE, {vr, static_cast<uint64_t>(rnd(0, 7)), t});
    CHECK(q[1] == sto::ST_OK && bitsd(q[2]) >= 0.0);
    const uint64_t filt = static_cast<uint64_t>(rnd(0, 3));
    q = call(sto::OP_VOUCH_LIST, {vr, filt, static_cast<uint64_t>(rnd(0, 7)), t, 0, 64, 0});
    CHECK(q[1] == sto::ST_OK && q[2] <= v.edges.size());
    if (filt == 0) {
      CHECK(q[2] == v.edges.size());
      const uint64_t* b = reinterpret_cast<const uint64_t*>(core->bulk_ptr(0, 8 * 8 * 64));
      for (size_t k = 0; k < v.edges.size() && k < 64; ++k) CHECK(static_cast<int32_t>(b[8 * k]) == v.edges[k]);
    }
    if (!v.edges.empty()) {
      const int32_t e = pick(v.edges);
      q = call(sto::OP_EDGE_READ, {static_cast<uint64_t>(e)});
      CHECK(q[1] == sto::ST_OK && static_cast<int32_t>(q[9]) == v.row);
      if (rnd(0, 3) == 0) CHECK(call(sto::OP_RELEASE_BOND, {static_cast<uint64_t>(e), t})[1] == sto::ST_OK);
    }
    q = call(sto::OP_EDGE_READ, {static_cast<uint64_t>(bad_index(T().cap.E))});
    CHECK(q[1] == sto::ST_BAD_ARG);
    q = call(sto::OP_RELEASE_BOND, {static_cast<uint64_t>(bad_index(T().cap.E)), t});
    CHECK(q[1] == sto::ST_BAD_ARG);
  }
  void slash() {
    if (vss.empty()) return;
    FzVs& v = pick(vss);
    std::vector<uint64_t> pairs;
    for (int a = 0; a < 8; ++a) {
      pairs.push_back(static_cast<uint64_t>(a));
      pairs.push_back(dbits(rndf()));
    }
    const uint64_t off = static_cast<uint64_t>(core->stage_raw(reinterpret_cast<const uint8_t*>(pairs.data()),
                                                               8 * pairs.size()));
    const uint64_t* q = call(sto::OP_SLASH, {static_cast<uint64_t>(v.row), static_cast<uint64_t>(rnd(0, 7)),
                                             dbits(rndf()), dbits(rndf()), static_cast<uint64_t>(now), 8, off, 0, 4096,
                                             65536, static_cast<uint64_t>(rnd(0, 2))});
    CHECK(q[1] == sto::ST_OK && q[3] >= 8);
    if (rnd(0, 2) == 0) {
      q = call(sto::OP_RELEASE_SESSION, {static_cast<uint64_t>(v.row), static_cast<uint64_t>(now)});
      CHECK(q[1] == sto::ST_OK && q[2] <= v.edges.size());
    }
  }
  void retire() {
    if (vss.empty()) return;
    const size_t i = static_cast<size_t>(rnd(0, static_cast<int>(vss.size()) - 1));
    FzVs& v = vss[i];
    const uint64_t* q = call(sto::OP_V_RETIRE, {static_cast<uint64_t>(v.row), 0, 1024});
    CHECK(q[1] == sto::ST_OK && q[2] == v.edges.size());
    const uint64_t* b = reinterpret_cast<const uint64_t*>(core->bulk_ptr(0, 24 * 1024));
    for (size_t k = 0; k < v.edges.size(); ++k) {
      CHECK(static_cast<int32_t>(b[3 * k]) == v.edges[k]);
      core->release_row(sto::RK_E, v.edges[k]);
    }
    v.edges.clear();
    if (rnd(0, 1)) {
      core->release_row(sto::RK_V, v.row);
      vss.erase(vss.begin() + static_cast<std::ptrdiff_t>(i));
    }
    CHECK(call(sto::OP_V_RETIRE, {static_cast<uint64_t>(bad_index(T().cap.V)), 0, 16})[1] == sto::ST_BAD_ARG);
  }

  // ------------------------------------------------------------- sagas
  void saga() {
    if (sagas.empty() || rnd(0, 5) == 0) {
      const int64_t g = row(sto::RK_G, 'G');
      CHECK(call(sto::OP_SAGA_CREATE, {static_cast<uint64_t>(g), static_cast<uint64_t>(now)})[1] == sto::ST_OK);
      sagas.push_back(FzSaga{g, SG_RUNNING, {}, {}});
      CHECK(call(sto::OP_SAGA_CREATE, {static_cast<uint64_t>(g), 0})[1] == sto::ST_BAD_STATE);
      return;
    }
    FzSaga& g = pick(sagas);
    const uint64_t gr = static_cast<uint64_t>(g.row);
    switch (rnd(0, 5)) {
      case 0: {
        if (g.steps.size() >= 12) break;
        const int64_t s = row(sto::RK_T, 'T');
        CHECK(call(sto::OP_STEP_ADD, {gr, static_cast<uint64_t>(s), 1, 2})[1] == sto::ST_OK);
        g.steps.push_back(static_cast<int32_t>(s));
        g.sstate.push_back(ST_PENDING);
        break;
      }
      case 1: {
        if (g.steps.empty()) break;
        const size_t k = static_cast<size_t>(rnd(0, static_cast<int>(g.steps.size()) - 1));
        const uint8_t to = static_cast<uint8_t>(rnd(0, 6));
        const uint64_t* q = call(sto::OP_STEP_TRANSITION, {static_cast<uint64_t>(g.steps[k]), to,
                                                           static_cast<uint64_t>(now), ~0ull});
        const bool ok = (step_transitions(g.sstate[k]) >> to) & 1u;
        CHECK(q[1] == (ok ? sto::ST_OK : sto::ST_BAD_STATE) && q[2] == g.sstate[k]);
        if (ok) g.sstate[k] = to;
        break;
      }
      case 2: {
        if (g.steps.empty()) break;
        const size_t k = static_cast<size_t>(rnd(0, static_cast<int>(g.steps.size()) - 1));
        const uint8_t to = static_cast<uint8_t>(rnd(0, 6));
        CHECK(call(sto::OP_STEP_SET, {static_cast<uint64_t>(g.steps[k]), to, 1})[1] == sto::ST_OK);
        g.sstate[k] = to;
        const uint64_t* q = call(sto::OP_STEP_READ, {static_cast<uint64_t>(g.steps[k])});
        CHECK(q[1] == sto::ST_OK && q[2] == to && q[3] == 1 && static_cast<int64_t>(q[6]) == g.row);
        break;
      }
      case 3: {
        const uint8_t to = static_cast<uint8_t>(rnd(0, 4));
        const uint64_t* q = call(sto::OP_SAGA_TRANSITION, {gr, to, static_cast<uint64_t>(now)});
        const bool ok = (saga_transitions(g.state) >> to) & 1u;
        CHECK(q[1] == (ok ? sto::ST_OK : sto::ST_BAD_STATE));
        if (ok) g.state = to;
        break;
      }
      case 4: {
        const bool plan = rnd(0, 1);
        const uint64_t* q = call_list(plan ? sto::OP_SAGA_PLAN : sto::OP_SAGA_READ, {gr, g.steps.size(), 0, 0}, 2,
                                      g.steps);
        CHECK(q[1] == sto::ST_OK && q[2] == g.state && q[5] == g.steps.size());
        if (plan) {
          uint64_t m = 0;
          for (uint8_t x : g.sstate) m += x == ST_COMMITTED;
          CHECK(q[6] == m);
        }
        break;
      }
      default:  // release the saga and its steps
        release_saga(static_cast<size_t>(&g - sagas.data()));
    }
  }
  void bad_saga_args() {
    const sto::Tables& t = T();
    const uint64_t bg = static_cast<uint64_t>(bad_index(t.cap.G)), bt = static_cast<uint64_t>(bad_index(t.cap.T));
    CHECK(call(sto::OP_STEP_TRANSITION, {bt, 1, 0, ~0ull})[1] == sto::ST_BAD_ARG);
    CHECK(call(sto::OP_STEP_SET, {bt, 1, ~0ull})[1] == sto::ST_BAD_ARG);
    CHECK(call(sto::OP_STEP_READ, {bt})[1] == sto::ST_BAD_ARG);
    CHECK(call(sto::OP_SAGA_TRANSITION, {bg, 1, 0})[1] == sto::ST_BAD_ARG);
    CHECK(call(sto::OP_SAGA_CREATE, {bg, 0})[1] == sto::ST_BAD_ARG);
    CHECK(call(sto::OP_STEP_ADD, {bg, 0, 0, 0})[1] == sto::ST_BAD_ARG);
    const std::vector<int32_t> one{static_cast<int32_t>(bt)};
    CHECK(call_list(sto::OP_SAGA_READ, {sagas.empty() ? bg : static_cast<uint64_t>(sagas[0].row), 1, 0, 0}, 2, one)[1] ==
          sto::ST_BAD_ARG);
    CHECK(call_list(sto::OP_SAGA_PLAN, {bg, 0, 0, 0}, 2, {})[1] == sto::ST_BAD_ARG);
  }

  // ------------------------------------------------------------- rows
  void bad_free_rows() {  // out-of-range rows and unknown kinds are refused; no live row is touched
    const sto::Tables& t = T();
    const uint64_t kind = static_cast<uint64_t>(rnd(0, 7));
    const int64_t caps[] = {t.cap.S, t.cap.G, t.cap.T, t.cap.E, t.cap.D, t.cap.V, 1, 1};
    std::vector<int32_t> idx;
    const int n = rnd(1, 120);
    for (int k = 0; k < n; ++k) idx.push_back(static_cast<int32_t>(bad_index(caps[kind])));
    CHECK(call_list(sto::OP_FREE_ROWS, {kind, idx.size(), 0}, 2, idx)[1] == sto::ST_BAD_ARG);
  }
  void control() {
    const uint32_t ops[] = {sto::OP_NOP, sto::OP_FLUSH, sto::OP_ACQUIRE, sto::OP_STOP};
    CHECK(call(ops[rnd(0, 3)], {})[1] == sto::ST_OK);
    core->drain();
  }

  // ------------------------------------------------------------- template batch
  // reserve_deltas + alloc_rows, then the template pipeline's host twin writes
  // whole sessions into the same tables the commands use.
  void template_batch() {
    const int n = rnd(1, 40), D = rnd(0, 8), nch = rnd(0, 4);
    std::vector<int32_t> srow(n), grow_(n), trow(n);
    while (!core->alloc_rows_raw(sto::RK_S, n, srow.data())) grow('S');
    while (!core->alloc_rows_raw(sto::RK_G, n, grow_.data())) grow('G');
    while (!core->alloc_rows_raw(sto::RK_T, n, trow.data())) grow('T');
    std::vector<int32_t> caps(static_cast<size_t>(n * D), 1024 + 64 * nch), drow(caps.size());
    std::vector<int64_t> doff(caps.size());
    for (int tries = 0; !caps.empty(); ++tries) {
      const int rc = core->reserve_deltas_raw(caps.data(), caps.size(), drow.data(), doff.data());
      if (rc == 0) break;
      CHECK(tries < 8);
      if (tries >= 8) return;
      if (rc == -3) {
        core->grow_payload(2 * core->payload_cap() + 2048 * static_cast<int64_t>(caps.size()));
        ++grows_B;
      } else if (core->reclaim_pool(sto::RK_D) == 0) {
        grow('D');
      }
    }
    for (int32_t x : srow)
      if (std::find(freed_s.begin(), freed_s.end(), x) != freed_s.end()) ++reused;
    std::vector<int32_t> sagent(n), status(n, -1);
    for (auto& x : sagent) x = rnd(0, kAgents - 1);
    std::vector<unsigned long long> stats(kStatSpread * kPipeStats, 0);
    TemplateArgs a{};
    a.t = T();
    a.n = n;
    a.slot = srow.data();
    a.gslot = grow_.data();
    a.tslot = trow.data();
    a.drow = drow.data();
    a.doff = doff.data();
    a.session_agent = sagent.data();
    a.agent_id = agent_id.data();
    a.agent_pool = agent_pool.data();
    a.agent_sigma = agent_sigma.data();
    a.changes = changes.data();
    a.pool = StrPool{pool.bytes.data(), pool.off.data(), pool.len.data()};
    a.deltas = D;
    a.nch = nch;
    a.creator = kAgents;
    a.maxpart = 10;
    a.minsig = 0.5;
    a.audit = 1;
    a.t0 = now;
    a.seed = 99;
    a.id_base = id_base;
    a.gc_retention_us = 1000;
    a.status = status.data();
    a.stats = stats.data();
    a.id_stride = 1;
    id_base += static_cast<uint64_t>(n);
    HostTeeSink sink;
    for (int64_t i = 0; i < n; ++i) {
      const PipeCounters c = template_session(a, i, sink);
      for (int k = 0; k < kPipeStats; ++k) stats[k] += c.v[k];
    }
    CHECK(stats[0] == static_cast<unsigned long long>(n));
    const sto::Tables& t = T();
    for (int i = 0; i < n; ++i) {
      const int64_t s = srow[i];
      FzSess f{s, sto::row_stamp(t, s), t.s_state[s], 10, 0.5};
      f.sid = "tmpl";
      CHECK(t.s_state[s] == SS_ARCHIVED && t.s_dcount[s] == D);
      if (status[i] == TP_OK) {
        f.agents.push_back(sagent[i]);
        f.active.push_back(1);
        f.pactive = 1;
      } else {
        CHECK(status[i] == TP_JOIN);  // σ below min_sigma_eff: the reference's join refusal
        CHECK(t.s_pcount[s] == 0);
      }
      for (int d = 0; d < D; ++d) f.drows.push_back(drow[static_cast<size_t>(i * D + d)]);
      bool ok;
      const std::vector<uint32_t> lv = chain(f, &ok);
      CHECK(ok);
      if (t.s_commit_n[s] == D && D > 0) {
        const std::vector<uint32_t> root = merkle_of(lv);
        CHECK(std::memcmp(root.data(), t.s_root + 8 * s, 32) == 0);
      }
      sess.push_back(f);
      sagas.push_back(FzSaga{grow_[i], t.g_state[grow_[i]], {trow[i]}, {t.t_state[trow[i]]}});
      CHECK(t.t_state[trow[i]] == ST_COMMITTED);
    }
    template_sessions += n;
  }

  void release_saga(size_t i) {
    for (int32_t s : sagas[i].steps) core->release_row(sto::RK_T, s);
    core->release_row(sto::RK_G, sagas[i].row);
    sagas.erase(sagas.begin() + static_cast<std::ptrdiff_t>(i));
  }

  void step() {
    // bounded working set: old rows go back to the allocator (and are reused)
    while (sess.size() > 120) release_session();
    while (sagas.size() > 120) release_saga(static_cast<size_t>(rnd(0, static_cast<int>(sagas.size()) - 1)));
    switch (rnd(0, 29)) {
      case 0: case 1: case 2: create(); break;
      case 3: create_on_live(); break;
      case 4: case 5: case 6: join(); break;
      case 7: leave(); break;
      case 8: tweak(); break;
      case 9: case 10: lifecycle(); break;
      case 11: bad_session_args(); break;
      case 12: case 13: case 14: capture(); break;
      case 15: bad_capture(); break;
      case 16: merkle(); break;
      case 17: verify(); break;
      case 18: delta_read(); break;
      case 19: reads(); break;
      case 20: close(); break;
      case 21: case 22: release_session(); break;
      case 23: vouch(); break;
      case 24: liability_reads(); slash(); break;
      case 25: retire(); break;
      case 26: saga(); saga(); break;
      case 27: bad_saga_args(); bad_free_rows(); break;
      case 28: control(); break;
      default: if (rnd(0, 3) == 0) template_batch(); else create();
    }
  }
};

static void test_store_programs() {
  for (uint64_t seed : {1ull, 2ull, 3ull}) {
    StoreFuzz f(seed);
    f.run(4000);
    std::printf("store programs seed %llu: grows S%d D%d E%d B%d, %d reused rows, %d template sessions\n",
                static_cast<unsigned long long>(seed), f.grows_S, f.grows_D, f.grows_E, f.grows_B, f.reused,
                f.template_sessions);
  }
}

// Ring mode of the template pipeline (GovernanceEngine's private store): rows
// addressed (slot_base + i) % ring, records at fixed arena offsets, each wrap
// evicting the previous occupant, plus the N08 event ring and the device cursor.
static void test_store_template() {
  Pool pool;
  const int A = 9;
  std::vector<int32_t> apool, aid;
  std::vector<double> asig;
  for (int a = 0; a < A; ++a) {
    apool.push_back(pool.add("did:mesh:ring-" + std::to_string(a)));
    aid.push_back(a);
    asig.push_back(0.55 + 0.045 * a);
  }
  std::vector<ChangeIds> ch;
  for (int d = 0; d < 8; ++d) ch.push_back(ChangeIds{pool.add("/r" + std::to_string(d)), pool.add("add"), pool.add("x"), -1});
  const int ring = 50, D = 5, rec = 1024;
  sto::Caps c{ring, 2, ring * 8, 4, 1, ring, ring, 4096, static_cast<int64_t>(ring) * 8 * rec + 4096};
  HostCols cols;
  cols.resize(c);
  StoreCore core(-1, cols.ptrs(), c, 8, 1 << 16, 1 << 16, 0, 0);
  const int64_t evcap = 8 * kStatSpread * 64;
  std::vector<uint8_t> etype(evcap);
  std::vector<int32_t> eslot(evcap), eagent(evcap), eaux(evcap);
  std::vector<int64_t> ets(evcap);
  std::vector<unsigned long long> ecur(kStatSpread, 0);
  std::vector<int64_t> cursor{0, 0, 1'767'225'600'000'000LL};
  std::vector<int32_t> sagent(ring);
  for (int i = 0; i < ring; ++i) sagent[i] = i % A;
  std::vector<int32_t> status(ring);
  uint64_t total_events = 0;
  for (int launch = 0; launch < 3; ++launch) {
    const int n = launch == 1 ? ring : 37;
    TemplateArgs a{};
    a.t = core.tables();
    a.n = n;
    a.session_agent = sagent.data();
    a.agent_id = aid.data();
    a.agent_pool = apool.data();
    a.agent_sigma = asig.data();
    a.changes = ch.data();
    a.pool = StrPool{pool.bytes.data(), pool.off.data(), pool.len.data()};
    a.deltas = D;
    a.nch = 1;
    a.creator = A;
    a.maxpart = 4;
    a.minsig = 0.5;
    a.audit = 1;
    a.seed = 5;
    a.gc_retention_us = 1;
    a.status = status.data();
    a.ring_cap = ring;
    a.dstride = 8;
    a.rec_bytes = rec;
    a.off_base = 4096;
    a.id_stride = 3;
    a.cursor = cursor.data();
    a.ev = EventRing{etype.data(), eslot.data(), eagent.data(), ets.data(), eaux.data(), ecur.data(), evcap};
    HostTeeSink sink;
    for (int64_t i = 0; i < n; ++i) {
      const PipeCounters pc = template_session(a, i, sink);
      const int seg = static_cast<int>((i / 64) % kStatSpread);
      const unsigned long long first = ecur[seg];
      const sto::Tables& t = core.tables();
      const uint32_t ne = template_event_count(pc, t.s_terminated[template_rows(a, i).s] != 0);
      ecur[seg] += ne;
      total_events += ne;
      template_events(a, i, pc, [&](uint32_t k, int64_t slot, const EventRec& e) {
        event_store(a.ev, seg, first + k, static_cast<int32_t>(slot), e);
      });
    }
    const sto::Tables& t = core.tables();
    for (int i = 0; i < n; ++i) {
      const int64_t s = (cursor[0] + i) % ring;
      CHECK(status[i] == TP_OK && t.s_state[s] == SS_ARCHIVED && t.s_dcount[s] == D);
      // re-derive the chain from the arena and compare the stored root
      std::vector<uint32_t> lv;
      const uint32_t* prev = nullptr;
      for (int d = 0; d < D; ++d) {
        const int64_t dr = s * 8 + d;
        CHECK(t.d_sess[dr] == s && t.d_turn[dr] == d + 1 && t.d_off[dr] == 4096 + dr * rec);
        std::vector<uint8_t> b(static_cast<size_t>(t.d_len[dr]));
        core.payload_read(t.d_off[dr], t.d_len[dr], b.data());
        if (t.d_hole[dr] >= 0) put_hex(b.data() + t.d_hole[dr], prev);
        uint32_t h[8];
        sto::sha256_mem(b.data(), b.size(), h);
        CHECK(std::memcmp(h, t.d_hash + 8 * dr, 32) == 0);
        lv.insert(lv.end(), h, h + 8);
        prev = t.d_hash + 8 * dr;
      }
      CHECK(std::memcmp(merkle_of(lv).data(), t.s_root + 8 * s, 32) == 0);
      // the same rows answer the store's own commands
      std::vector<int32_t> idx;
      for (int d = 0; d < D; ++d) idx.push_back(static_cast<int32_t>(s * 8 + d));
      const uint64_t* q = core.wait(core.post_raw(sto::OP_DELTA_MERKLE, std::vector<uint64_t>{static_cast<uint64_t>(s), static_cast<uint64_t>(D), 0}.data(), 3,
                                                  reinterpret_cast<const uint8_t*>(idx.data()), 4 * idx.size()));
      CHECK(q[1] == sto::ST_OK);
      for (int k = 0; k < 8; ++k) CHECK(q[3 + k] == t.s_root[8 * s + k]);
    }
    cursor[0] = (cursor[0] + n) % ring;
    cursor[1] += 3 * n;
    cursor[2] += 100;
  }
  CHECK(total_events > 0);
  unsigned long long stored = 0;
  for (int sgi = 0; sgi < kStatSpread; ++sgi) stored += std::min<unsigned long long>(ecur[sgi], evcap / kStatSpread);
  CHECK(stored <= static_cast<unsigned long long>(evcap));
}

int main() {
  test_hashing();
  test_sagas();
  test_liability();
  test_governance();
  test_session();
  test_store_programs();
  test_store_template();
  if (g_fail) {
    std::fprintf(stderr, "host_selftest: %d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host_selftest: all checks passed\n");
  return 0;
}
