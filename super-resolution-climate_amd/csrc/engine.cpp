// srmi engine: the RCAN / EDSR network plan, workspace layout and the
// forward / backward / optimizer orchestration behind the C ABI of
// include/srmi.h.  Every launch is asynchronous on the caller's stream; the
// engine never synchronises and allocates nothing (graph-capturable).
//
// Network structure follows the reference exactly:
//   RCAN  sres/model/rcan/network.py:7-77, blocks.py:58-76
//   EDSR  sres/model/edsr/network.py:9-32, common/residual.py:26-50,
//         common/upsample.py:32-66
// Parameter order = the reference state_dict order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "srmi_internal.hpp"

using namespace srmi;

namespace {

struct ConvRef {
  long long w = -1, b = -1;  // param offsets
  int cin = 0, cout = 0, ps = 0;
  long long f_off = -1, d_off = -1, pb_off = -1;  // pack offsets (MFMA convs only)
};

struct RCABRef {
  ConvRef c1, c2;
  long long ca_w1, ca_b1, ca_w2, ca_b2;
};

struct Plan {
  srmi_model_config cfg;
  std::vector<srmi_param_info> params;
  long long n_params = 0;
  ConvRef head, body_tail, tail;
  std::vector<std::vector<RCABRef>> groups;  // RCAN
  std::vector<ConvRef> group_tail;            // RCAN
  std::vector<ConvRef> res1, res2;            // EDSR
  std::vector<ConvRef> ups;
  std::vector<ConvRef*> mfma_convs;
  long long pack_elems = 0, pbias_elems = 0;
  int nups = 0;
};

long long add_param(Plan& P, std::initializer_list<int> shape) {
  srmi_param_info pi{};
  pi.offset = P.n_params;
  pi.ndim = (int)shape.size();
  long long n = 1;
  int k = 0;
  for (int s : shape) {
    pi.shape[k++] = s;
    n *= s;
  }
  pi.numel = n;
  P.params.push_back(pi);
  P.n_params += n;
  return pi.offset;
}

ConvRef add_conv(Plan& P, int cin, int cout, int k) {
  ConvRef c;
  c.cin = cin;
  c.cout = cout;
  c.w = add_param(P, {cout, cin, k, k});
  c.b = add_param(P, {cout});
  return c;
}

int build_plan(const srmi_model_config* cfg, Plan& P) {
  if (!cfg) return SRMI_ERR_ARG;
  const srmi_model_config& c = *cfg;
  if (c.nfeatures != 64) return SRMI_ERR_UNSUPPORTED;
  if (c.nchannels_in < 1 || c.nchannels_in > 4 || c.nchannels_out < 1 || c.nchannels_out > 4) return SRMI_ERR_UNSUPPORTED;
  if (c.scale != 2 && c.scale != 4 && c.scale != 8) return SRMI_ERR_UNSUPPORTED;
  if (c.nlayers < 1 || c.batch < 1 || c.lr_h < 4 || c.lr_w < 16) return SRMI_ERR_ARG;
  if (c.arch == SRMI_ARCH_RCAN && (c.nblocks < 1 || c.reduction < 1 || 64 % c.reduction)) return SRMI_ERR_ARG;
  // the CA kernels take CR = 64 / reduction in 4 .. 32, a multiple of 4 (records sized for 32):
  // refused here rather than at the first CA launch
  if (c.arch == SRMI_ARCH_RCAN && (64 / c.reduction > 32 || (64 / c.reduction) % 4)) return SRMI_ERR_UNSUPPORTED;
  if (c.arch != SRMI_ARCH_RCAN && c.arch != SRMI_ARCH_EDSR) return SRMI_ERR_ARG;
  if (c.dtype != SRMI_DTYPE_BF16 && c.dtype != SRMI_DTYPE_F32) return SRMI_ERR_ARG;
  if (c.flags & ~(SRMI_FLAG_NO_RCAB_INFER | SRMI_FLAG_CA_PASS | SRMI_FLAG_DU_PASS)) return SRMI_ERR_ARG;  // (retired bits refused)
  P = Plan();
  P.cfg = c;
  const int F = 64;
  P.head = add_conv(P, c.nchannels_in, F, 3);
  if (c.arch == SRMI_ARCH_RCAN) {
    P.groups.resize(c.nlayers);
    for (int g = 0; g < c.nlayers; ++g) {
      for (int b = 0; b < c.nblocks; ++b) {
        RCABRef r;
        r.c1 = add_conv(P, F, F, 3);
        r.c2 = add_conv(P, F, F, 3);
        r.ca_w1 = add_param(P, {F / c.reduction, F, 1, 1});
        r.ca_b1 = add_param(P, {F / c.reduction});
        r.ca_w2 = add_param(P, {F, F / c.reduction, 1, 1});
        r.ca_b2 = add_param(P, {F});
        P.groups[g].push_back(r);
      }
      P.group_tail.push_back(add_conv(P, F, F, 3));
    }
  } else {
    for (int i = 0; i < c.nlayers; ++i) {
      P.res1.push_back(add_conv(P, F, F, 3));
      P.res2.push_back(add_conv(P, F, F, 3));
    }
  }
  P.body_tail = add_conv(P, F, F, 3);
  P.nups = (int)std::lround(std::log2((double)c.scale));
  for (int k = 0; k < P.nups; ++k) {
    ConvRef u = add_conv(P, F, 4 * F, 3);
    u.ps = 1;
    P.ups.push_back(u);
  }
  P.tail = add_conv(P, F, c.nchannels_out, 3);
  // MFMA convs get filter packs in the operand type (bf16 or fp32)
  for (auto& grp : P.groups)
    for (auto& r : grp) {
      P.mfma_convs.push_back(&r.c1);
      P.mfma_convs.push_back(&r.c2);
    }
  for (auto& t : P.group_tail) P.mfma_convs.push_back(&t);
  for (size_t i = 0; i < P.res1.size(); ++i) {
    P.mfma_convs.push_back(&P.res1[i]);
    P.mfma_convs.push_back(&P.res2[i]);
  }
  P.mfma_convs.push_back(&P.body_tail);
  for (auto& u : P.ups) P.mfma_convs.push_back(&u);
  for (ConvRef* cr : P.mfma_convs) {
    const long long n = (long long)cr->cout * cr->cin * 9;
    cr->f_off = P.pack_elems;
    P.pack_elems += n;
    cr->d_off = P.pack_elems;
    P.pack_elems += n;
    cr->pb_off = P.pbias_elems;
    P.pbias_elems += cr->cout;
  }
  return 0;
}

// ---------------------------------------------------------------- workspace
struct Carver {
  size_t off = 0;
  char* base = nullptr;
  template <class T>
  T* take(size_t count) {
    off = (off + 255) & ~(size_t)255;
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += count * sizeof(T);
    return p;
  }
};

int choose_row_splits(int N, int H, int Cout, int cu_budget = 0) {
  // wgrad grid = N*rs chunks x Cout/64 (one workgroup per CU by LDS); aim at >= 3/4
  // of the CU budget while keeping as few partial slabs (N*rs) as possible; rows per
  // chunk % 4 == 0
  const int target = 3 * (cu_budget > 0 ? cu_budget : 256) / 4;
  int best = 1;
  for (int rs = 1; rs <= H / 4; ++rs) {
    if (H % rs || (H / rs) % 4) continue;
    best = rs;
    if (N * rs * (Cout / 64) >= target) break;
  }
  return best;
}

}  // namespace

struct srmi_engine {
  Plan P;
  int train = 0;
  // operand storage: bf16 (SRMI_DTYPE_BF16: bf16 MFMA operands, fp32 accumulation
  // and residual stream) or fp32 (SRMI_DTYPE_F32: exact fp32 everywhere).  The
  // activation / gradient-map / filter-pack pointers below are typed bf16_t* but
  // hold esz-byte elements; at() does their element arithmetic.
  int f32 = 0;
  size_t esz = 2;
  int N = 0, h = 0, w = 0, C = 0, Co = 0, S = 0;
  int cu_budget = 0;  // CUs one launch aims to fill (0 = all)
  size_t mapn = 0;  // elements of one [N][h][w][64] map
  // forward state
  float *X0f, *Rf, *Hf;
  bf16_t* HB;    // hb maps
  int n_hb;      // number of hb slots
  bf16_t *T, *U; // train: [nl*nb] maps; infer: 1 each
  bf16_t* RESb;
  bf16_t* PS[3];  // pixel-shuffle outputs (scale s: [N][h*2^k][w*2^k][64])
  float *rec, *brec;
  float *ppool, *pacc;
  float* mpart;  // conv1's partial CA means [N][runs per image <= nstrips][64] (SRMI_CA_MPART)
  // backward
  float *GAf, *GBf, *dRESf;
  bf16_t *GAb, *GBb, *DU, *DZ, *dRESb;
  bf16_t* dPS[3];
  float *slab, *bslab;
  size_t slab_floats, bslab_floats;
  // the RCAB filter gradients' slab sets of one residual group: set (b, c) = RCAB b's conv2
  // (c = 0) / conv1 (c = 1) filter gradient, b = 1 .. nblocks; (0, 0) the group tail's.  One
  // per launch, so the reductions can wait for the group's end (one launch for all)
  std::vector<float*> slab_sets, bslab_sets;
  size_t slab_r_floats = 0, bslab_r_floats = 0;
  // (SRMI_F2_MLP 0: the reductions ride in the next launch pair's CA-backward launch, so two
  //  sets per conv alternate -- RCAB b by the parity of b, the group tail the other parity of
  //  RCAB nblocks' -- and only four sets are ever touched)
  int slab_idx(int b, int c) const {
    if (SRMI_F2_MLP) return b * 2 + c;
    const int q = b == 0 ? ((P.cfg.nblocks & 1) ^ 1) : (b & 1);
    return (q + 1) * 2 + c;  // (sets 2 .. 5: the group tail's own (0, 1) slot is never allocated)
  }
  float* slab_r(int b, int c) const { return slab_sets[slab_idx(b, c)]; }
  float* bslab_r(int b, int c) const { return bslab_sets[slab_idx(b, c)]; }
  float* lpart;
  int lpart_n;
  float* zeros;  // 256 zero bytes (DMA padding source)
  // packs
  bf16_t* packs;
  float* pbias;
  PackEntry* d_entries;
  long long* d_caoffs;
  std::vector<PackEntry> h_entries;
  std::vector<long long> h_caoffs;
  int max_cob = 0, max_cib = 0;  // largest Cout / 64, Cin / 64 of the packed convs
  bool tables_uploaded = false;
  int last_n = 0;
  // the backward stage srmi_backward_stages must run next (0 after a forward or a
  // completed backward): the gradient-stream buffers and the slab parity carry over
  // from one stage to the next, so a skipped, repeated or reordered stage is refused
  int next_stage = 0;
  const float* probe_prm = nullptr;  // the parameters of the last backward / inference forward (srmi_engine_probe)

  bf16_t* at(bf16_t* base, size_t elems) const {
    return reinterpret_cast<bf16_t*>(reinterpret_cast<char*>(base) + elems * esz);
  }
  bf16_t* hb(int g, int b) const {
    const int nb1 = P.cfg.arch == SRMI_ARCH_RCAN ? P.cfg.nblocks + 1 : 1;
    const int k = g * nb1 + b;
    return at(HB, (size_t)(train ? k : (k % n_hb)) * mapn);
  }
  int nbe() const { return P.cfg.arch == SRMI_ARCH_RCAN ? P.cfg.nblocks : 1; }
  bf16_t* Tm(int g, int b) const { return train ? at(T, (size_t)(g * nbe() + (b - 1)) * mapn) : T; }
  bf16_t* Um(int g, int b) const { return train ? at(U, (size_t)(g * P.cfg.nblocks + (b - 1)) * mapn) : U; }
  float* recp(int g, int b) const {
    return train ? rec + (size_t)(g * P.cfg.nblocks + (b - 1)) * N * 160 : rec;
  }
  float* brecp(int g, int b) const { return brec + (size_t)(g * P.cfg.nblocks + (b - 1)) * N * 224; }
};

// bf16 partial slabs for the RCAB filter gradients (tuning.hpp).  The other filter
// gradients (group / body tails, upsamplers: 26 launches per step) keep fp32 slabs:
// bf16 there measured +0.3 % (noise) and doubled the split dependence of their sums
// (one engine of 16 tiles vs 2 x 2 engines of 4: 2.4e-4 rel-L2 of the gradient)
constexpr bool kSlab16 = SRMI_SLAB16 != 0;

// The RCAB filter gradients run beside their dgrad convs (one fused launch, the
// CU budget split in halves), so their row chunks are sized for HALF the engine's
// budget: fewer, longer chunks write fewer partial slabs (at C2 2 x 24-row chunks
// per image instead of 3 x 16).
static int engine_cus(const srmi_engine* e) { return e->cu_budget > 0 ? e->cu_budget : 256; }
// CU shares of the two parts of a fused launch, in percent of the engine budget taken
// by the filter gradient: after the ReLU-mask dgrad of conv2 (FUSE_WG2) and after the
// gradient-accumulating dgrad of conv1 (FUSE_WG1, the heavier conv epilogue)
static int fuse_wg_cus(const srmi_engine* e, int which) {
  (void)which;  // half the budget for both fused launches (44 / 56 % measured within noise)
  return engine_cus(e) / 2;
}
static int rcab_row_splits(const srmi_engine* e, int n, int which) {
  return choose_row_splits(n, e->h, 64, fuse_wg_cus(e, which));
}

static size_t carve(srmi_engine* e, char* base) {
  Carver cv;
  cv.base = base;
  auto act = [&](size_t count) { return reinterpret_cast<bf16_t*>(cv.take<char>(count * e->esz)); };
  const Plan& P = e->P;
  const int N = e->N;
  const size_t m = e->mapn;
  const bool rcan = P.cfg.arch == SRMI_ARCH_RCAN;
  const int nl = P.cfg.nlayers, nb = rcan ? P.cfg.nblocks : 0;
  e->X0f = cv.take<float>(m);
  e->Rf = cv.take<float>(m);
  e->Hf = cv.take<float>(m);
  const int nslots = rcan ? nl * (nb + 1) + 1 : nl + 1;
  e->n_hb = e->train ? nslots : 3;
  e->HB = act(m * e->n_hb);
  const int nconv1 = rcan ? nl * nb : nl;
  e->T = act(m * (e->train ? nconv1 : 1));
  e->U = rcan ? act(m * (e->train ? nconv1 : 1)) : nullptr;
  e->RESb = act(m);
  for (int k = 0; k < 3; ++k) e->PS[k] = nullptr;
  for (int k = 0; k < P.nups; ++k) e->PS[k] = act(m << (2 * (k + 1)));
  const int nstrips = conv3x3_nstrips(e->h, e->w);
  if (rcan) {
    e->rec = cv.take<float>((size_t)(e->train ? nl * nb : 1) * N * 160);
    e->brec = e->train ? cv.take<float>((size_t)nl * nb * N * 224) : nullptr;  // [N][160] + dm[N][64]
    e->ppool = cv.take<float>((size_t)N * nstrips * 64);
    e->mpart = e->train ? cv.take<float>((size_t)N * nstrips * 64) : nullptr;
    e->pacc = cv.take<float>((size_t)N * nstrips * 128);
  }
  e->lpart_n = 1024;
  e->lpart = cv.take<float>(e->lpart_n);
  e->zeros = cv.take<float>(64);
  if (e->train) {
    e->GAf = cv.take<float>(m);
    e->GBf = cv.take<float>(m);
    e->dRESf = cv.take<float>(m);
    e->GAb = act(m);
    e->GBb = act(m);
    e->DU = act(m);
    e->DZ = act(m);
    e->dRESb = act(m);
    for (int k = 0; k < 3; ++k) e->dPS[k] = nullptr;
    for (int k = 0; k < P.nups; ++k) e->dPS[k] = act(m << (2 * (k + 1)));
    // slab: max over all wgrads
    size_t sf = 0, bf = 0;
    auto upd = [&](int H, int W, int Cout) {
      // a call may pass fewer tiles than the capacity (a short last batch), and
      // fewer tiles get more row splits: size for the largest n * rs(n)
      for (int n = 1; n <= N; ++n) {
        const size_t ns = (size_t)n * choose_row_splits(n, H, Cout, e->cu_budget) * (W % 48 == 0 ? W / 48 : 1);
        sf = std::max(sf, ns * Cout * 576);
        bf = std::max(bf, ns * Cout);
      }
    };
    upd(e->h, e->w, 64);
    for (int k = 0; k < P.nups; ++k) upd(e->h << k, e->w << k, 256);
    // head / tail slabs
    const int Hs = e->h * e->S;
    sf = std::max(sf, (size_t)N * (e->h / 2) * 64 * (9 * e->C + 1));  // head wgrad: 2-row bands
    sf = std::max(sf, (size_t)N * (Hs / 4) * e->Co * 577);  // tail_wgrad: 4-row bands
    e->slab_floats = sf;
    e->bslab_floats = bf;
    e->slab = cv.take<float>(sf);
    e->bslab = cv.take<float>(bf);
    if (rcan) {  // the RCAB filter-gradient slab sets (64-channel convs only)
      size_t ns = 0;  // (wgrad48: a slab per 48-wide column tile too, as wgrad3x3_nslabs counts)
      for (int n = 1; n <= N; ++n)
        ns = std::max(ns, (size_t)n * std::max(rcab_row_splits(e, n, 1), rcab_row_splits(e, n, 2)) *
                              (e->w % 48 == 0 ? e->w / 48 : 1));
      e->slab_r_floats = ns * 64 * 576;
      e->bslab_r_floats = ns * 64;
      const int nsets = SRMI_F2_MLP ? (P.cfg.nblocks + 1) * 2 : 6;  // (slab_idx)
      e->slab_sets.assign(nsets, nullptr);
      e->bslab_sets.assign(nsets, nullptr);
      for (int i = 0; i < nsets; ++i) {
        if (i == 1) continue;  // (the group tail has one filter gradient)
        e->slab_sets[i] = cv.take<float>(e->slab_r_floats);
        e->bslab_sets[i] = cv.take<float>(e->bslab_r_floats);
      }
    }
  }
  e->packs = act(P.pack_elems);
  e->pbias = cv.take<float>(P.pbias_elems);
  e->d_entries = cv.take<PackEntry>(P.mfma_convs.size());
  e->d_caoffs = cv.take<long long>((size_t)std::max(1, nl * nb) * 5);
  return cv.off + 256;
}

static int init_engine(srmi_engine* e, const srmi_model_config* cfg, int train) {
  int rc = build_plan(cfg, e->P);
  if (rc) return rc;
  e->train = train;
  e->f32 = cfg->dtype == SRMI_DTYPE_F32;
  e->esz = e->f32 ? 4 : 2;
  e->N = cfg->batch;
  e->h = cfg->lr_h;
  e->w = cfg->lr_w;
  e->C = cfg->nchannels_in;
  e->Co = cfg->nchannels_out;
  e->S = cfg->scale;
  e->cu_budget = cfg->cu_budget > 0 ? cfg->cu_budget : 0;
  e->mapn = (size_t)e->N * e->h * e->w * 64;
  if (e->h % 4 || (e->w % 32 && e->w % 48)) return SRMI_ERR_SHAPE;
  const int Hs = e->h * e->S;
  if (Hs % 16 || ((e->w * e->S) % 32)) return SRMI_ERR_SHAPE;
  // the kernels store activation / gradient maps through buffer resources with a
  // 32-bit byte range: refuse any map of 2^32 bytes or more (the largest is the
  // last pixel-shuffle output, mapn << 2 nups elements, and the fp32 streams)
  const size_t lim = (size_t)1 << 32;
  const size_t ps_bytes = (e->mapn << (2 * e->P.nups)) * e->esz;
  const size_t f32_bytes = e->mapn * 4;
  const size_t hr_bytes = (size_t)e->N * std::max(e->C, e->Co) * Hs * (e->w * e->S) * 4;
  if (ps_bytes >= lim || f32_bytes >= lim || hr_bytes >= lim) return SRMI_ERR_SHAPE;
  return 0;
}

static void build_tables(srmi_engine* e) {
  e->h_entries.clear();
  e->max_cob = e->max_cib = 0;
  for (ConvRef* c : e->P.mfma_convs) {
    PackEntry pe{};
    pe.w_off = c->w;
    pe.b_off = c->b;
    pe.f_off = c->f_off;
    pe.d_off = c->d_off;
    pe.pb_off = c->pb_off;
    pe.Cout = c->cout;
    pe.Cin = c->cin;
    pe.ps = c->ps;
    e->h_entries.push_back(pe);
    e->max_cob = std::max(e->max_cob, (c->cout + 63) / 64);
    e->max_cib = std::max(e->max_cib, (c->cin + 63) / 64);
  }
  e->h_caoffs.clear();
  for (auto& grp : e->P.groups)
    for (auto& r : grp) {
      e->h_caoffs.push_back(r.ca_w1);
      e->h_caoffs.push_back(r.ca_b1);
      e->h_caoffs.push_back(r.ca_w2);
      e->h_caoffs.push_back(r.ca_b2);
      e->h_caoffs.push_back(r.c2.b);
    }
}

static inline hipStream_t S_(void* s) { return reinterpret_cast<hipStream_t>(s); }

// --------------------------------------------------------------- conv helpers
// forward convs sized for this share of the engine's CU budget (A/B: fewer, longer runs)
static ConvParams fwd_params(srmi_engine* e, const ConvRef& c, const bf16_t* x, int n, int H, int W, bf16_t* yb,
                             float* yf, const float* r1, float* part, float alpha) {
  ConvParams p{};
  p.x = x;
  p.w = e->at(e->packs, c.f_off);
  p.bias = e->pbias + c.pb_off;
  p.f32 = e->f32;
  p.N = n;
  p.H = H;
  p.W = W;
  p.Cin = c.cin;
  p.Cout = c.cout;
  p.in_mode = IN_PLAIN;
  p.yb = yb;
  p.yf = yf;
  p.r1 = r1;
  p.part = part;
  p.part_stride = 64;
  p.alpha = alpha;
  p.zeros = e->zeros;
  p.cu_budget = e->cu_budget;
  return p;
}

static int conv_fwd(srmi_engine* e, const ConvRef& c, const bf16_t* x, int n, int H, int W, int epi, bf16_t* yb,
                    float* yf, const float* r1, float* part, float alpha, hipStream_t st) {
  return conv3x3_launch(fwd_params(e, c, x, n, H, W, yb, yf, r1, part, alpha), epi, st);
}

// dgrad of conv c: input dy (Cout channels, PS layout if c.ps), output Cin channels
static ConvParams dgrad_params(srmi_engine* e, const ConvRef& c, const bf16_t* dy, int n, int H, int W, int* epi,
                               bf16_t* yb, float* yf, const float* r1, const float* r2, const float* r3,
                               const bf16_t* aux, float* part, float alpha, const bf16_t* r1b = nullptr) {
  ConvParams p{};
  p.x = dy;
  p.w = e->at(e->packs, c.d_off);
  p.bias = nullptr;
  p.f32 = e->f32;
  p.N = n;
  p.H = H;
  p.W = W;
  p.Cin = c.cout;
  p.Cout = c.cin;
  p.in_mode = c.ps ? IN_UNSHUF : IN_PLAIN;
  p.yb = yb;
  p.yf = yf;
  p.r1 = r1;
  p.r1b = r1b;
  p.r2 = r2;
  p.r3 = r3;
  p.aux = aux;
  p.part = part;
  p.part_stride = 128;
  p.alpha = alpha;
  p.zeros = e->zeros;
  p.cu_budget = e->cu_budget;
  // the hot RCAB cases: specialised epilogues without runtime operand checks
  if (*epi == EPI_DG_ACC && r1 && aux && part && !yb && !r2 && !r3 && yf && c.cout == 64 && !c.ps)
    *epi = EPI_DG_ACC_CA;
  if (*epi == EPI_DG_ACC && r1b && !r1 && aux && part && yb && !r2 && !r3 && !yf && c.cout == 64 && !c.ps)
    *epi = EPI_DG_ACC_CA16;  // (the bf16 engine's in-group gradient stream)
  if (*epi == EPI_DG_ACC && !r1b && !r1 && aux && part && yb && !r2 && !r3 && !yf && c.cout == 64 && !c.ps)
    *epi = EPI_DG_CA16;  // (the group tail's dgrad: the stream's start)
  if (*epi == EPI_DG_ACC && r1b && !r1 && !aux && !part && yb && yf && r2 && c.cout == 64 && !c.ps)
    *epi = EPI_DG_ACC_G1;  // (the group's first RCAB: the stream's end)
  return p;
}

static int conv_dgrad(srmi_engine* e, const ConvRef& c, const bf16_t* dy, int n, int H, int W, int epi, bf16_t* yb,
                      float* yf, const float* r1, const float* r2, const float* r3, const bf16_t* aux, float* part,
                      float alpha, hipStream_t st) {
  ConvParams p = dgrad_params(e, c, dy, n, H, W, &epi, yb, yf, r1, r2, r3, aux, part, alpha);
  return conv3x3_launch(p, epi, st);
}

// filter gradient of conv c into `slab`/`bslab` (capacity cap/bcap floats); the
// reduction into grads is returned in *red
static int wgrad_params(srmi_engine* e, const ConvRef& c, const bf16_t* x, const bf16_t* dy, int n, int H, int W,
                        float* grads, bool with_bias, float alpha, int row_splits, float* slab, float* bslab,
                        size_t cap, size_t bcap, WgradParams* out, ReduceSet* red, bool slab16 = false) {
  WgradParams p{};
  p.x = x;
  p.dy = dy;
  p.f32 = e->f32;
  p.N = n;
  p.H = H;
  p.W = W;
  p.Cout = c.cout;
  p.dy_mode = c.ps ? IN_UNSHUF : IN_PLAIN;
  p.imgs_per_wg = 1;
  p.row_splits = row_splits;
  p.slab = slab;
  p.bslab = bslab;
  p.zeros = e->zeros;
  // bf16 weight slabs only where the wgrad48 body writes them (layout 1)
  p.slab16 = slab16 && !e->f32 && wgrad3x3_slab_layout(p) == 1;
  const size_t ns = (size_t)wgrad3x3_nslabs(p);
  if (ns * c.cout * 576 > cap || ns * c.cout > bcap) return SRMI_ERR_WORKSPACE;
  *out = p;
  *red = ReduceSet{p.slab, p.bslab, (int)ns, c.cout, c.ps, wgrad3x3_slab_layout(p), alpha, grads + c.w,
                   with_bias ? grads + c.b : nullptr, p.slab16};
  return 0;
}

// filter gradient + its reduction, both on st (upsampler / group-tail / body-tail /
// EDSR convs)
static int conv_wgrad(srmi_engine* e, const ConvRef& c, const bf16_t* x, const bf16_t* dy, int n, int H, int W,
                      float* grads, bool with_bias, float alpha, hipStream_t st) {
  WgradParams p;
  ReduceSet r;
  const int rc = wgrad_params(e, c, x, dy, n, H, W, grads, with_bias, alpha, choose_row_splits(n, H, c.cout, e->cu_budget),
                              e->slab, e->bslab, e->slab_floats, e->bslab_floats, &p, &r);
  if (rc) return rc;
  const int rc2 = wgrad3x3_launch(p, st);
  if (rc2) return rc2;
  return wgrad_reduce_launch(r.slab, r.bslab, r.nslab, r.Cout, r.ps, r.layout, r.alpha, r.gw, r.gb, st, r.slab16);
}

// a dgrad conv and the filter gradient of the same conv (independent, both reading
// dy): one fused launch where the shapes allow (bf16, 48-wide tiles), else the two
// launches one after the other on the same stream
static int dgrad_with_wgrad(srmi_engine* e, const ConvParams& cp, int epi, const WgradParams& wp, int which,
                            hipStream_t st) {
  if (rcab_bwd_fusable(cp, wp)) return rcab_bwd_launch(cp, epi, engine_cus(e) - fuse_wg_cus(e, which), wp, st);
  const int rc = wgrad3x3_launch(wp, st);
  if (rc) return rc;
  return conv3x3_launch(cp, epi, st);
}

// SRMI_TRACE_ERRORS=1 in the environment: every failing step prints its line
static int trace_rc(int rc, int line) {
  static const bool on = std::getenv("SRMI_TRACE_ERRORS") != nullptr;
  if (on) std::fprintf(stderr, "srmi: engine.cpp:%d -> %d\n", line, rc);
  return rc;
}
#define RC(x)                                  \
  do {                                         \
    int _rc = (x);                             \
    if (_rc) return trace_rc(_rc, __LINE__);   \
  } while (0)
#define HC(x)                                  \
  do {                                         \
    const hipError_t _he = (x);                \
    if (_he != hipSuccess) return -(int)_he;   \
  } while (0)

static int upload_tables(srmi_engine* e, hipStream_t st) {
  if (e->tables_uploaded) return 0;
  build_tables(e);
  hipError_t err = hipMemcpyAsync(e->d_entries, e->h_entries.data(), e->h_entries.size() * sizeof(PackEntry),
                                  hipMemcpyHostToDevice, st);
  if (err != hipSuccess) return -(int)err;
  if (!e->h_caoffs.empty()) {
    err = hipMemcpyAsync(e->d_caoffs, e->h_caoffs.data(), e->h_caoffs.size() * sizeof(long long),
                         hipMemcpyHostToDevice, st);
    if (err != hipSuccess) return -(int)err;
  }
  err = hipMemsetAsync(e->zeros, 0, 256, st);
  if (err != hipSuccess) return -(int)err;
  // the host vectors must outlive the async copies: keep them in the engine
  e->tables_uploaded = true;
  return 0;
}

// inference (no saved activations): each RCAB as one launch with a workgroup per image
// (rcab_infer.hip) -- bf16, 48-wide tiles, a CA bottleneck the MLP code handles
static bool use_rcab_infer(const srmi_engine* e) {
  const int CR = 64 / e->P.cfg.reduction;
  return !(e->P.cfg.flags & SRMI_FLAG_NO_RCAB_INFER) && !e->train && !e->f32 &&
         e->P.cfg.arch == SRMI_ARCH_RCAN && e->w == 48 && e->h % 4 == 0 && CR >= 4 && CR <= 32 && CR % 4 == 0;
}

// training forward: the CA forward of an RCAB (CALayer, sres/model/rcan/network.py:
// 31-47, 61-64) without a pass of its own.  conv1 writes t and its per-strip sums
// (EPI_RELU_POOL); conv2 (EPI_CA_RESID_U) stores u for backward and adds s bf16(u) into
// the residual pair in its epilogue, with s = the CA MLP of mean(u), and mean(u) from t's
// statistics and conv2's bf16 filter image (ca_scale.hpp), computed by every conv2
// workgroup in its prologue (1; its own launch between the convs measured -2.5 %).
// 0: conv1, conv2 + pool writing u, the CA pass (ca_fwd) -- the exact-fp32 mode and tiles
// other than 48 wide always run this form; SRMI_FLAG_CA_PASS selects it at run time.
// bf16, 48-wide tiles, a bottleneck the scale code handles.
static int ca_fwd_mode(const srmi_engine* e) {
  const int CR = 64 / e->P.cfg.reduction;
  if (!e->train || e->f32 || e->P.cfg.arch != SRMI_ARCH_RCAN || e->w != 48 || e->h % 4 || CR < 4 || CR > 32 ||
      CR % 4 || (e->P.cfg.flags & SRMI_FLAG_CA_PASS))
    return 0;
  return SRMI_CA_FWD;
}

// ------------------------------------------------------------------ forward
static int forward_impl(srmi_engine* e, const float* prm, const float* lr, float* sr, int n, hipStream_t st) {
  const Plan& P = e->P;
  const int h = e->h, w = e->w, HW = h * w;
  const int nstrips = conv3x3_nstrips(h, w);
  RC(head_fwd_launch(lr, prm + P.head.w, prm + P.head.b, n, e->C, h, w, e->X0f, e->hb(0, 0), e->f32, st));
  if (P.cfg.arch == SRMI_ARCH_RCAN) {
    const int nl = P.cfg.nlayers, nb = P.cfg.nblocks, R = P.cfg.reduction;
    for (int g = 0; g < nl; ++g) {
      const float* rin = g == 0 ? e->X0f : e->Rf;
      for (int b = 1; b <= nb; ++b) {
        const RCABRef& r = P.groups[g][b - 1];
        if (use_rcab_infer(e)) {  // inference: the RCAB as one launch, a workgroup per image
          uint8_t* lo = reinterpret_cast<uint8_t*>(e->Hf);  // the pair's lo8 remainder, 1 B / element
          const ConvParams c1 = fwd_params(e, r.c1, e->hb(g, b - 1), n, h, w, e->Tm(g, b), nullptr, nullptr, nullptr, 1.f);
          const ConvParams c2 = fwd_params(e, r.c2, e->Tm(g, b), n, h, w, e->Um(g, b), nullptr, nullptr, e->ppool, 1.f);
          RC(rcab_infer_launch(c1, c2, e->ppool, nstrips, prm + r.ca_w1, prm + r.ca_b1, prm + r.ca_w2, prm + r.ca_b2,
                               64 / R, b == 1 ? rin : nullptr, b == 1 ? nullptr : e->hb(g, b - 1),
                               b == 1 ? nullptr : lo, e->hb(g, b), lo, e->recp(g, b), st));
          continue;
        }
        if (ca_fwd_mode(e)) {  // training: the CA forward inside conv2
          uint8_t* lo = reinterpret_cast<uint8_t*>(e->Hf);  // the pair's lo8 remainder (as below)
          ConvParams c1 = fwd_params(e, r.c1, e->hb(g, b - 1), n, h, w, e->Tm(g, b), nullptr, nullptr, e->ppool, 1.f);
          ConvParams c2 = fwd_params(e, r.c2, e->Tm(g, b), n, h, w, e->Um(g, b), nullptr, b == 1 ? rin : nullptr,
                                     nullptr, 1.f);
          // SRMI_CA_MPART: conv1's workgroups leave their share of the CA mean (the matvec
          // on conv2's bf16 filter image) for conv2, which then reads no t border lines
          const int nruns = SRMI_CA_MPART ? conv64_runs_per_image(c1) : 0;
          if (SRMI_CA_MPART) {
            c1.cas.mpart = e->mpart;
            c1.cas.nruns = nruns;
            c1.cas.wimg = c2.w;
            c1.cas_on = 1;
          }
          RC(conv3x3_launch(c1, EPI_RELU_POOL, st));
          c2.r1h = b == 1 ? nullptr : e->hb(g, b - 1);
          c2.r1l = b == 1 ? nullptr : lo;
          c2.yph = e->hb(g, b);
          c2.ypl = lo;
          const CaScale cas{e->Tm(g, b), e->ppool, nstrips, prm + r.ca_w1, prm + r.ca_b1, prm + r.ca_w2,
                            prm + r.ca_b2, e->pbias + r.c2.pb_off, 64 / R, e->recp(g, b)};
          c2.cas = cas;
          if (SRMI_CA_MPART) {
            c2.cas.mpart = e->mpart;
            c2.cas.nruns = nruns;
          }
          c2.cas_on = 1;
          RC(conv3x3_launch(c2, EPI_CA_RESID_U, st));
          continue;
        }
        RC(conv_fwd(e, r.c1, e->hb(g, b - 1), n, h, w, EPI_RELU_BF16, e->Tm(g, b), nullptr, nullptr, nullptr, 1.f, st));
        RC(conv_fwd(e, r.c2, e->Tm(g, b), n, h, w, EPI_POOL_BF16, e->Um(g, b), nullptr, nullptr, e->ppool, 1.f, st));
        if (e->f32) {
          RC(ca_fwd_launch(e->Um(g, b), e->ppool, nstrips, prm + r.ca_w1, prm + r.ca_b1, prm + r.ca_w2, prm + r.ca_b2,
                           n, HW, 64, R, b == 1 ? rin : e->Hf, e->Hf, e->hb(g, b), e->recp(g, b), 1, st));
        } else {
          // the residual stream inside the group as the pair hb (bf16, the next conv's
          // input) + lo (the 8-bit lo8 remainder, 1 B per element, in Hf's memory):
          // 16 significant bits per element (common.hpp); the group input rin is fp32
          uint8_t* lo = reinterpret_cast<uint8_t*>(e->Hf);
          RC(ca_fwd_launch(e->Um(g, b), e->ppool, nstrips, prm + r.ca_w1, prm + r.ca_b1, prm + r.ca_w2, prm + r.ca_b2,
                           n, HW, 64, R, b == 1 ? rin : nullptr, nullptr, e->hb(g, b), e->recp(g, b), 0, st,
                           b == 1 ? nullptr : e->hb(g, b - 1), b == 1 ? nullptr : lo, lo));
        }
      }
      RC(conv_fwd(e, P.group_tail[g], e->hb(g, nb), n, h, w, EPI_RESID, e->hb(g + 1, 0), e->Rf, rin, nullptr, 1.f,
                  st));
    }
    RC(conv_fwd(e, P.body_tail, e->hb(nl, 0), n, h, w, EPI_RESID, e->RESb, nullptr, e->X0f, nullptr, 1.f, st));
  } else {
    const int nl = P.cfg.nlayers;
    for (int i = 0; i < nl; ++i) {
      const float* rin = i == 0 ? e->X0f : e->Rf;
      RC(conv_fwd(e, P.res1[i], e->hb(i, 0), n, h, w, EPI_RELU_BF16, e->Tm(i, 1), nullptr, nullptr, nullptr, 1.f, st));
      RC(conv_fwd(e, P.res2[i], e->Tm(i, 1), n, h, w, EPI_RESID, e->hb(i + 1, 0), e->Rf, rin, nullptr,
                  P.cfg.res_scale, st));
    }
    RC(conv_fwd(e, P.body_tail, e->hb(nl, 0), n, h, w, EPI_RESID, e->RESb, nullptr, e->X0f, nullptr, 1.f, st));
  }
  const bf16_t* cur = e->RESb;
  int H = h, W = w;
  for (int k = 0; k < P.nups; ++k) {
    RC(conv_fwd(e, P.ups[k], cur, n, H, W, EPI_PS_BF16, e->PS[k], nullptr, nullptr, nullptr, 1.f, st));
    cur = e->PS[k];
    H *= 2;
    W *= 2;
  }
  RC(tail_fwd_launch(cur, prm + P.tail.w, prm + P.tail.b, n, e->Co, H, W, sr, e->f32, st));
  e->last_n = n;
  e->next_stage = 0;
  if (!e->train) e->probe_prm = prm;  // (srmi_engine_probe which = 3)
  return 0;
}

// ----------------------------------------------------------------- backward
// Stages of the RCAN backward, in order: 0 = tail conv, upsamplers and body tail;
// 1 .. nlayers = residual groups nlayers-1 .. 0; nlayers + 1 = the head.  backward_impl
// runs stages s_lo .. s_hi (EDSR: all of them at once), so that a caller can enqueue a
// group's gradient all-reduce right behind that group (srmi_backward_stages).
static int backward_stages(const srmi_engine* e) { return e->P.cfg.arch == SRMI_ARCH_RCAN ? e->P.cfg.nlayers + 2 : 1; }

// The CALayer backward inside the fused conv2 backward (ca_bwd.hpp; SRMI_FLAG_DU_PASS off):
// the bf16 engine, a fusable 48-wide launch, CR = 64 / reduction in 4 .. 32 and a multiple
// of 4 (the MLP's thread mapping).  Else the CA backward is a launch of its own.
static bool du_in_f2(const srmi_engine* e, const ConvParams& cp, const WgradParams& wp, int epi) {
  const int CR = 64 / e->P.cfg.reduction;
  return !e->f32 && !(e->P.cfg.flags & SRMI_FLAG_DU_PASS) && rcab_bwd_du_from_g() && epi == EPI_DG_RELUMASK &&
         rcab_bwd_fusable(cp, wp) && CR % 4 == 0 && CR >= 4 && CR <= 32;
}

static int backward_impl(srmi_engine* e, const float* prm, const float* lr, const float* sr, const float* hr,
                         const float* loss4, const float* dy, float* grads, void** group_events, hipStream_t st,
                         int s_lo = 0, int s_hi = 1 << 30) {
  const Plan& P = e->P;
  const int n = e->last_n, h = e->h, w = e->w, HW = h * w;
  const int nstrips = conv3x3_nstrips(h, w);
  int H = h << P.nups, W = w << P.nups;
  e->probe_prm = prm;
  const bool rcan = P.cfg.arch == SRMI_ARCH_RCAN;
  if (!rcan) {
    s_lo = 0;
    s_hi = 1 << 30;
  }
  const int nl = P.cfg.nlayers;
  if (s_lo <= 0) {
    // tail conv 64 -> C
    const bf16_t* xlast = e->PS[P.nups - 1];
    const float* yv = dy ? dy : sr;
    const float* tv = dy ? nullptr : hr;
    const float* lv = dy ? nullptr : loss4;
    RC(tail_dgrad_launch(yv, tv, lv, prm + P.tail.w, n, e->Co, H, W, e->dPS[P.nups - 1], e->f32, st));
    int nsl = 0;
    RC(tail_wgrad_launch(yv, tv, lv, xlast, n, e->Co, H, W, e->slab, &nsl, e->f32, st));
    RC(tail_wgrad_reduce_launch(e->slab, nsl, e->Co, grads + P.tail.w, grads + P.tail.b, st));
    // upsamplers, last to first
    for (int k = P.nups - 1; k >= 0; --k) {
      H /= 2;
      W /= 2;
      const bf16_t* xin = k == 0 ? e->RESb : e->PS[k - 1];
      RC(conv_wgrad(e, P.ups[k], xin, e->dPS[k], n, H, W, grads, true, 1.f, st));
      if (k > 0)
        RC(conv_dgrad(e, P.ups[k], e->dPS[k], n, H, W, EPI_PLAIN_BF16, e->dPS[k - 1], nullptr, nullptr, nullptr,
                      nullptr, nullptr, nullptr, 1.f, st));
      else
        RC(conv_dgrad(e, P.ups[k], e->dPS[k], n, H, W, EPI_DG_ACC, e->dRESb, e->dRESf, nullptr, nullptr, nullptr,
                      nullptr, nullptr, 1.f, st));
    }
  }
  // body tail: res = conv(hb_last) + x0
  float *gRf = e->GAf, *ghf = e->GBf;
  bf16_t *gRb = e->GAb, *ghb = e->GBb;
  if (rcan) {
    const int nb = P.cfg.nblocks, R = P.cfg.reduction;
    if (s_lo <= 0) {
      RC(conv_wgrad(e, P.body_tail, e->hb(nl, 0), e->dRESb, n, h, w, grads, true, 1.f, st));
      RC(conv_dgrad(e, P.body_tail, e->dRESb, n, h, w, EPI_DG_ACC, gRb, gRf, nullptr, nullptr, nullptr, nullptr,
                    nullptr, 1.f, st));
    }
    // One stream, two launches per RCAB:
    //   [the CA backward (MLP, du from g in LDS) -> dgrad conv2 -> dz || filter gradient conv2 (t, du)]
    //   [dgrad conv1 -> g (+ CA sums of the next RCAB)  ||  filter gradient conv1 (hb, dz)]
    // (SRMI_FLAG_DU_PASS, exact fp32, unfusable shapes: a CA-backward launch writing du
    // first).  The filter gradients write their RCAB's slab sets, reduced by one launch at
    // the group's end, before the group's event.
    const int rs2 = rcab_row_splits(e, n, 2), rs1 = rcab_row_splits(e, n, 1);
    // the gradient stream INSIDE a residual group (w.r.t. every RCAB output): bf16 in the
    // bf16 engine, in the buffer of the group input gradient's bf16 copy (ghb: the group's
    // first RCAB reads it and overwrites it in place with that copy), fp32 (ghf) in the
    // exact-fp32 engine.  The group input gradient itself stays fp32.
    const bool g16 = !e->f32;
    for (int g = nl - 1; g >= 0; --g) {
      const int stage = nl - g;
      // the gradient streams swap after every group: the state group g starts from
      const bool sw = ((nl - 1 - g) & 1) != 0;
      gRf = sw ? e->GBf : e->GAf;
      ghf = sw ? e->GAf : e->GBf;
      gRb = sw ? e->GBb : e->GAb;
      ghb = sw ? e->GAb : e->GBb;
      if (stage < s_lo || stage > s_hi) continue;
      const ConvRef& gt = P.group_tail[g];
      // the filter-gradient reductions: collected for one launch at the group's end (or, with
      // the CA backward's MLP as a launch of its own (SRMI_F2_MLP 0), riding in that launch)
      ReduceSet prev2{}, prev1{};
      bool have_prev = false;
      std::vector<ReduceSet> group_sets;
      auto defer_prev = [&]() {
        if (!have_prev) return;
        if (prev2.gw || prev2.gb) group_sets.push_back(prev2);
        if (prev1.gw || prev1.gb) group_sets.push_back(prev1);
        have_prev = false;
      };
      // group tail: its dgrad (the bf16 stream's start, with the CA sums of RCAB nb) and its
      // filter gradient as one fused launch, like the RCABs' (slab set (0, 0), reduced with the
      // RCABs'), else (exact fp32, unfusable shapes) the two launches and the reduction in turn
      {
        int epi = EPI_DG_ACC;
        const ConvParams cp = dgrad_params(e, gt, gRb, n, h, w, &epi, g16 ? ghb : nullptr, g16 ? nullptr : ghf,
                                           nullptr, nullptr, nullptr, e->Um(g, nb), e->pacc, 1.f);
        WgradParams wp{};
        if (g16)
          RC(wgrad_params(e, gt, e->hb(g, nb), gRb, n, h, w, grads, true, 1.f, rs1, e->slab_r(0, 0),
                          e->bslab_r(0, 0), e->slab_r_floats, e->bslab_r_floats, &wp, &prev2));
        if (g16 && rcab_bwd_fusable(cp, wp)) {
          RC(dgrad_with_wgrad(e, cp, epi, wp, 1, st));
          prev1 = ReduceSet{};  // (no second reduction: gw = gb = null)
          prev1.Cout = prev2.Cout;
          have_prev = true;
        } else {
          RC(conv_wgrad(e, gt, e->hb(g, nb), gRb, n, h, w, grads, true, 1.f, st));
          RC(conv3x3_launch(cp, epi, st));
        }
      }
      for (int b = nb; b >= 1; --b) {
        const RCABRef& r = P.groups[g][b - 1];
        bf16_t* du = e->DU;
        bf16_t* dz = e->DZ;
        ReduceSet red2, red1;
        WgradParams wp;
        int epi = EPI_DG_RELUMASK;
        ConvParams cp = dgrad_params(e, r.c2, du, n, h, w, &epi, dz, nullptr, nullptr, nullptr, nullptr, e->Tm(g, b),
                                     nullptr, 1.f);
        RC(wgrad_params(e, r.c2, e->Tm(g, b), du, n, h, w, grads, false, 1.f, rs2, e->slab_r(b, 0), e->bslab_r(b, 0),
                        e->slab_r_floats, e->bslab_r_floats, &wp, &red2, kSlab16));
        // The CALayer backward inside the fused conv2 backward (both its roles run the
        // image's MLP in their prologue and form du = bf16(g s + dm / HW) from the bf16
        // stream on their input rings; ca_bwd.hpp), or as a launch of its own writing du
        // (SRMI_FLAG_DU_PASS, exact fp32, unfusable shapes) that the conv2 backward reads
        const bool du_fused = du_in_f2(e, cp, wp, epi);
        if (du_fused) {
          cp.x = wp.dy = ghb;
          cp.gx = wp.gx = CaBwdIn{e->pacc, nstrips, e->recp(g, b), prm + r.ca_w1, prm + r.ca_w2, 64 / R,
                                  e->brecp(g, b), n, 1.f / (float)HW, SRMI_F2_MLP};
          if (SRMI_F2_MLP) {
            defer_prev();
          } else {  // the MLP launch (brec, dm), the previous pair's reductions riding in it
            RC(ca_bwd_du_launch(ghb, 1, e->pacc, nstrips, e->recp(g, b), prm + r.ca_w1, prm + r.ca_w2, n, HW, 64, R,
                                nullptr, e->brecp(g, b), 0, st, have_prev ? &prev2 : nullptr,
                                have_prev ? &prev1 : nullptr));
            have_prev = false;
          }
        } else if (SRMI_F2_MLP) {  // (its reductions, too, at the group's end: the default path's sums)
          defer_prev();
          RC(ca_bwd_du_launch(g16 ? static_cast<const void*>(ghb) : ghf, g16, e->pacc, nstrips, e->recp(g, b),
                              prm + r.ca_w1, prm + r.ca_w2, n, HW, 64, R, du, e->brecp(g, b), e->f32, st, nullptr,
                              nullptr));
        } else {  // (the reductions riding, as the default path's MLP launch carries them)
          RC(ca_bwd_du_launch(g16 ? static_cast<const void*>(ghb) : ghf, g16, e->pacc, nstrips, e->recp(g, b),
                              prm + r.ca_w1, prm + r.ca_w2, n, HW, 64, R, du, e->brecp(g, b), e->f32, st,
                              have_prev ? &prev2 : nullptr, have_prev ? &prev1 : nullptr));
          have_prev = false;
        }
        RC(dgrad_with_wgrad(e, cp, epi, wp, 2, st));
        const bool last = (b == 1);
        epi = EPI_DG_ACC;
        // g += dgrad(dz): in the group's first RCAB into the group input gradient (fp32 +
        // its bf16 copy, with the group's skip gradient gR), else the in-group stream
        if (g16)
          cp = dgrad_params(e, r.c1, dz, n, h, w, &epi, ghb, last ? ghf : nullptr, nullptr, last ? gRf : nullptr,
                            (last && g == 0) ? e->dRESf : nullptr, last ? nullptr : e->Um(g, b - 1),
                            last ? nullptr : e->pacc, 1.f, ghb);
        else
          cp = dgrad_params(e, r.c1, dz, n, h, w, &epi, last ? ghb : nullptr, ghf, ghf, last ? gRf : nullptr,
                            (last && g == 0) ? e->dRESf : nullptr, last ? nullptr : e->Um(g, b - 1),
                            last ? nullptr : e->pacc, 1.f);
        RC(wgrad_params(e, r.c1, e->hb(g, b - 1), dz, n, h, w, grads, true, 1.f, rs1, e->slab_r(b, 1),
                        e->bslab_r(b, 1), e->slab_r_floats, e->bslab_r_floats, &wp, &red1, kSlab16));
        RC(dgrad_with_wgrad(e, cp, epi, wp, 1, st));
        prev2 = red2;
        prev1 = red1;
        have_prev = true;
      }
      defer_prev();
      if (!group_sets.empty()) RC(wgrad_reduce_sets_launch(group_sets.data(), (int)group_sets.size(), st));
      // per-RCAB slots of recp / brecp (N x 160 and N x 224 floats at any CR <= 32)
      RC(ca_param_grads_batched_launch(e->recp(g, 1), e->brecp(g, 1), nb, n, (size_t)e->N * 160, (size_t)e->N * 224,
                                       64, R, e->d_caoffs + (size_t)g * nb * 5, grads, st));
      // the group's gradients are final here (one stream): the hook for a bucketed
      // all-reduce overlapped with the rest of backward
      if (group_events && group_events[g]) HC(hipEventRecord(reinterpret_cast<hipEvent_t>(group_events[g]), st));
    }
    // after all nl groups: the group-0 input gradient (the head's upstream)
    gRf = (nl & 1) ? e->GBf : e->GAf;
  } else {
    const float rsc = P.cfg.res_scale;
    RC(conv_wgrad(e, P.body_tail, e->hb(nl, 0), e->dRESb, n, h, w, grads, true, 1.f, st));
    RC(conv_dgrad(e, P.body_tail, e->dRESb, n, h, w, EPI_DG_ACC, gRb, gRf, nullptr, nullptr, nullptr, nullptr, nullptr,
                  1.f, st));
    for (int i = nl - 1; i >= 0; --i) {
      // block i: out = rsc * (conv2(relu(conv1(x)))) + x, grad wrt out = gR
      RC(conv_wgrad(e, P.res2[i], e->Tm(i, 1), gRb, n, h, w, grads, true, rsc, st));
      RC(conv_dgrad(e, P.res2[i], gRb, n, h, w, EPI_DG_RELUMASK, e->DZ, nullptr, nullptr, nullptr, nullptr,
                    e->Tm(i, 1), nullptr, rsc, st));
      RC(conv_wgrad(e, P.res1[i], e->hb(i, 0), e->DZ, n, h, w, grads, true, 1.f, st));
      RC(conv_dgrad(e, P.res1[i], e->DZ, n, h, w, EPI_DG_ACC, ghb, ghf, gRf, i == 0 ? e->dRESf : nullptr, nullptr,
                    nullptr, nullptr, 1.f, st));
      std::swap(gRf, ghf);
      std::swap(gRb, ghb);
    }
  }
  // head: only the weight gradient (the input gradient is never read)
  if (s_hi >= (rcan ? nl + 1 : 0)) {
    int nsl = 0;
    RC(head_wgrad_launch(lr, gRf, n, e->C, h, w, e->slab, &nsl, st));
    RC(head_wgrad_reduce_launch(e->slab, nsl, e->C, grads + P.head.w, grads + P.head.b, st));
  }
  return 0;
}

// =================================================================== C ABI
extern "C" {

int srmi_version(void) { return 200; }

int srmi_param_count(const srmi_model_config* cfg, long long* n_params, int* n_tensors) {
  Plan P;
  RC(build_plan(cfg, P));
  if (n_params) *n_params = P.n_params;
  if (n_tensors) *n_tensors = (int)P.params.size();
  return 0;
}

int srmi_param_table(const srmi_model_config* cfg, srmi_param_info* out, int cap) {
  Plan P;
  RC(build_plan(cfg, P));
  if (!out || cap < (int)P.params.size()) return SRMI_ERR_ARG;
  std::memcpy(out, P.params.data(), P.params.size() * sizeof(srmi_param_info));
  return (int)P.params.size();
}

int srmi_workspace_size(const srmi_model_config* cfg, int train, size_t* bytes) {
  srmi_engine e;
  RC(init_engine(&e, cfg, train));
  *bytes = carve(&e, nullptr);
  return 0;
}

int srmi_engine_create(const srmi_model_config* cfg, void* workspace, size_t ws_bytes, int train, srmi_engine** out) {
  if (!out || !workspace) return SRMI_ERR_ARG;
  srmi_engine* e = new (std::nothrow) srmi_engine();
  if (!e) return SRMI_ERR_ARG;
  int rc = init_engine(e, cfg, train);
  if (rc) {
    delete e;
    return rc;
  }
  const size_t need = carve(e, nullptr);
  if (ws_bytes < need) {
    delete e;
    return SRMI_ERR_WORKSPACE;
  }
  char* base = reinterpret_cast<char*>(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  if ((size_t)(base - (char*)workspace) + need - 256 > ws_bytes) {
    delete e;
    return SRMI_ERR_WORKSPACE;
  }
  carve(e, base);
  *out = e;
  return 0;
}

int srmi_engine_destroy(srmi_engine* e) {
  delete e;
  return 0;
}

int srmi_pack_weights(srmi_engine* e, const float* params, void* stream) {
  if (!e || !params) return SRMI_ERR_ARG;
  RC(upload_tables(e, S_(stream)));
  return pack_launch(params, e->d_entries, (int)e->h_entries.size(), e->max_cob, e->max_cib, e->packs, e->pbias,
                     e->f32, S_(stream));
}

int srmi_forward(srmi_engine* e, const float* params, const float* lr, float* sr, int n, void* stream) {
  if (!e || !params || !lr || !sr || n < 1 || n > e->N) return SRMI_ERR_ARG;
  if (!e->tables_uploaded) return SRMI_ERR_ARG;  // srmi_pack_weights first
  return forward_impl(e, params, lr, sr, n, S_(stream));
}

int srmi_backward(srmi_engine* e, const float* params, const float* lr, const float* sr, const float* hr,
                  const float* loss4, const float* dy, float* grads, void** group_events, void* stream) {
  if (!e || !e->train || !params || !lr || !grads || e->last_n < 1) return SRMI_ERR_ARG;
  if (!dy && (!sr || !hr || !loss4)) return SRMI_ERR_ARG;
  if (e->next_stage != 0) return SRMI_ERR_ARG;  // a staged backward is half-way through
  return backward_impl(e, params, lr, sr, hr, loss4, dy, grads, group_events, S_(stream));
}

int srmi_backward_stage_count(srmi_engine* e) { return e ? backward_stages(e) : SRMI_ERR_ARG; }

int srmi_backward_stages(srmi_engine* e, const float* params, const float* lr, const float* sr, const float* hr,
                         const float* loss4, const float* dy, float* grads, void** group_events, int first, int last,
                         void* stream) {
  if (!e || !e->train || !params || !lr || !grads || e->last_n < 1) return SRMI_ERR_ARG;
  if (!dy && (!sr || !hr || !loss4)) return SRMI_ERR_ARG;
  const int ns = backward_stages(e);
  if (first < 0 || last >= ns || first > last || (ns == 1 && (first != 0 || last != 0))) return SRMI_ERR_ARG;
  if (first != e->next_stage) return SRMI_ERR_ARG;  // stages run in order, each once per backward
  RC(backward_impl(e, params, lr, sr, hr, loss4, dy, grads, group_events, S_(stream), first, last));
  e->next_stage = last + 1 == ns ? 0 : last + 1;
  return 0;
}

int srmi_engine_probe(srmi_engine* e, int which, int reps, void* stream) {
  if (which == 3) {  // inference engines: the one-launch RCAB (0, 2) of the last forward
    if (!e || e->train || !use_rcab_infer(e) || e->last_n < 1 || reps < 1 || e->P.cfg.nblocks < 2)
      return SRMI_ERR_ARG;
    const int n = e->last_n, R = e->P.cfg.reduction;
    const RCABRef& r = e->P.groups[0][1];
    const float* prm = e->probe_prm;
    if (!prm) return SRMI_ERR_ARG;
    uint8_t* lo = reinterpret_cast<uint8_t*>(e->Hf);
    const ConvParams c1 = fwd_params(e, r.c1, e->hb(0, 1), n, e->h, e->w, e->Tm(0, 2), nullptr, nullptr, nullptr, 1.f);
    const ConvParams c2 = fwd_params(e, r.c2, e->Tm(0, 2), n, e->h, e->w, e->Um(0, 2), nullptr, nullptr, e->ppool, 1.f);
    for (int i = 0; i < reps; ++i)
      RC(rcab_infer_launch(c1, c2, e->ppool, conv3x3_nstrips(e->h, e->w), prm + r.ca_w1, prm + r.ca_b1,
                           prm + r.ca_w2, prm + r.ca_b2, 64 / R, nullptr, e->hb(0, 1), lo, e->hb(0, 2), lo,
                           e->recp(0, 2), S_(stream)));
    return 0;
  }
  if (which == 4) {  // does the backward form du inside the fused conv2 backward (1) or not (0)
    if (!e || !e->train || e->P.cfg.arch != SRMI_ARCH_RCAN || e->last_n < 1 || !e->probe_prm) return SRMI_ERR_ARG;
    const int n = e->last_n, b = e->P.cfg.nblocks >= 2 ? 2 : 1;
    const RCABRef& r = e->P.groups[0][b - 1];
    int epi = EPI_DG_RELUMASK;
    ConvParams cp = dgrad_params(e, r.c2, e->DU, n, e->h, e->w, &epi, e->DZ, nullptr, nullptr, nullptr, nullptr,
                                 e->Tm(0, b), nullptr, 1.f);
    WgradParams wp;
    ReduceSet red;
    RC(wgrad_params(e, r.c2, e->Tm(0, b), e->DU, n, e->h, e->w, e->slab, false, 1.f, rcab_row_splits(e, n, 2),
                    e->slab_r(b, 0), e->bslab_r(b, 0), e->slab_r_floats, e->bslab_r_floats, &wp, &red, kSlab16));
    return du_in_f2(e, cp, wp, epi) ? 1 : 0;
  }
  if (!e || !e->train || e->P.cfg.arch != SRMI_ARCH_RCAN || e->last_n < 1 || reps < 1) return SRMI_ERR_ARG;
  if (which != 1 && which != 2) return SRMI_ERR_ARG;
  const int n = e->last_n, h = e->h, w = e->w;
  const int b = e->P.cfg.nblocks >= 2 ? 2 : 1;
  const RCABRef& r = e->P.groups[0][b - 1];
  float* ghf = e->GBf;
  float* grads = e->slab;  // the reductions are not launched: any pointer
  WgradParams wp;
  ReduceSet red;
  ConvParams cp;
  int epi;
  if (which == 2) {
    epi = EPI_DG_RELUMASK;
    cp = dgrad_params(e, r.c2, e->DU, n, h, w, &epi, e->DZ, nullptr, nullptr, nullptr, nullptr, e->Tm(0, b), nullptr,
                      1.f);
    RC(wgrad_params(e, r.c2, e->Tm(0, b), e->DU, n, h, w, grads, false, 1.f, rcab_row_splits(e, n, 2),
                    e->slab_r(b, 0), e->bslab_r(b, 0), e->slab_r_floats, e->bslab_r_floats, &wp, &red, kSlab16));
    // (as backward_impl: the CA backward and du inside the fused launch; its record and dm
    //  go to brec, which the engine's next backward rewrites)
    if (e->probe_prm && du_in_f2(e, cp, wp, epi)) {
      cp.x = wp.dy = e->GBb;
      cp.gx = wp.gx = CaBwdIn{e->pacc, conv3x3_nstrips(h, w), e->recp(0, b), e->probe_prm + r.ca_w1,
                              e->probe_prm + r.ca_w2, 64 / e->P.cfg.reduction, e->brecp(0, b), n, 1.f / (float)(h * w),
                              SRMI_F2_MLP};
    }
  } else {
    const bool last = (b == 1);
    epi = EPI_DG_ACC;
    if (!e->f32)  // the bf16 in-group gradient stream, as backward_impl issues it
      cp = dgrad_params(e, r.c1, e->DZ, n, h, w, &epi, e->GBb, last ? ghf : nullptr, nullptr, last ? e->GAf : nullptr,
                        nullptr, last ? nullptr : e->Um(0, b - 1), last ? nullptr : e->pacc, 1.f, e->GBb);
    else
      cp = dgrad_params(e, r.c1, e->DZ, n, h, w, &epi, last ? e->GAb : nullptr, ghf, ghf, last ? e->GAf : nullptr,
                        nullptr, last ? nullptr : e->Um(0, b - 1), last ? nullptr : e->pacc, 1.f);
    RC(wgrad_params(e, r.c1, e->hb(0, b - 1), e->DZ, n, h, w, grads, true, 1.f, rcab_row_splits(e, n, 1),
                    e->slab_r(b, 1), e->bslab_r(b, 1), e->slab_r_floats, e->bslab_r_floats, &wp, &red, kSlab16));
  }
  for (int i = 0; i < reps; ++i) RC(dgrad_with_wgrad(e, cp, epi, wp, which, S_(stream)));
  return 0;
}

int srmi_rmse_partial(srmi_engine* e, const float* pred, const float* target, size_t n, double count_global,
                      float* loss4, void* stream) {
  if (!e || !pred || !target || !loss4) return SRMI_ERR_ARG;
  RC(sqerr_partial_launch(pred, target, n, e->lpart, e->lpart_n, S_(stream)));
  return sqerr_finish_launch(e->lpart, e->lpart_n, count_global, loss4, S_(stream));
}

int srmi_rmse_finalize(float* loss4, void* stream) {
  if (!loss4) return SRMI_ERR_ARG;
  return loss_finalize_launch(loss4, LOSS_RMSE, S_(stream));
}

int srmi_charbonnier_partial(srmi_engine* e, const float* pred, const float* target, size_t n, double count_global,
                             float eps, float* loss4, float* dy, void* stream) {
  if (!e || !pred || !target || (!loss4 && !dy) || count_global <= 0) return SRMI_ERR_ARG;
  RC(charb_partial_launch(pred, target, n, eps, count_global, dy, loss4 ? e->lpart : nullptr, e->lpart_n, S_(stream)));
  return loss4 ? sqerr_finish_launch(e->lpart, e->lpart_n, count_global, loss4, S_(stream)) : 0;
}

int srmi_loss_finalize(float* loss4, int kind, void* stream) {
  if (!loss4 || (kind != SRMI_LOSS_RMSE && kind != SRMI_LOSS_MEAN)) return SRMI_ERR_ARG;
  return loss_finalize_launch(loss4, kind, S_(stream));
}

int srmi_batch_losses(const float* pred, const float* target, int ntiles, long long tile_elems, int batch_size,
                      int kind, float eps, float* work, float* out, void* stream) {
  if (!pred || !target || !work || !out || (kind != SRMI_LOSS_RMSE && kind != SRMI_LOSS_MEAN)) return SRMI_ERR_ARG;
  return batch_losses_launch(pred, target, ntiles, tile_elems, batch_size, kind, eps, work, out, S_(stream));
}

int srmi_tile_loss_parts(const float* pred, const float* target, int ntiles, long long tile_elems, int kind,
                         float eps, float* parts, void* stream) {
  if (!pred || !target || !parts || (kind != SRMI_LOSS_RMSE && kind != SRMI_LOSS_MEAN)) return SRMI_ERR_ARG;
  return tile_loss_parts_launch(pred, target, ntiles, tile_elems, kind, eps, parts, S_(stream));
}

int srmi_loss_from_parts(const float* parts, int ntiles, double count_global, int kind, float* loss4, void* stream) {
  if (!parts || !loss4 || kind < -1 || kind > SRMI_LOSS_MEAN) return SRMI_ERR_ARG;
  return loss_from_parts_launch(parts, ntiles * kTileSub, count_global, kind, loss4, S_(stream));
}

int srmi_batch_loss_means(const float* sums, int ntiles, long long tile_elems, int batch_size, int kind, float* out,
                          void* stream) {
  if (!sums || !out || (kind != SRMI_LOSS_RMSE && kind != SRMI_LOSS_MEAN)) return SRMI_ERR_ARG;
  return batch_loss_means_launch(sums, ntiles, tile_elems, batch_size, kind, out, S_(stream));
}

int srmi_loss_combine(float* loss4, const float* parts4, int nparts, int kind, void* stream) {
  if (!loss4 || !parts4 || nparts < 1 || kind < -1 || kind > SRMI_LOSS_MEAN) return SRMI_ERR_ARG;
  return loss_combine_launch(loss4, parts4, nparts, kind, S_(stream));
}

int srmi_downsample(const float* hr, int N, int C, int H, int W, int scale, float* lr, void* stream) {
  return downsample_launch(hr, N, C, H, W, scale, lr, S_(stream));
}

int srmi_upsample(const float* lr, int N, int C, int h, int w, int scale, float* hr, void* stream) {
  return upsample_launch(lr, N, C, h, w, scale, hr, S_(stream));
}

int srmi_interpolate(const float* x, int N, int C, int H, int W, int Ho, int Wo, float rh, float rw, int mode, float* y,
                     void* stream) {
  return interp_launch(x, N, C, H, W, Ho, Wo, rh, rw, mode, y, S_(stream));
}

int srmi_adam_step(float* p, const float* g, float* m, float* v, size_t n, int step, float lr, float beta1,
                   float beta2, float eps, float weight_decay, void* stream) {
  if (step < 1) return SRMI_ERR_ARG;
  const double bc1 = 1.0 - std::pow((double)beta1, step);
  const double bc2 = 1.0 - std::pow((double)beta2, step);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)std::sqrt(bc2);
  return adam_launch(p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt, S_(stream));
}

// ---------------------------------------------------------------- op level
int srmi_conv3x3(const void* x, const void* wpack, const float* bias, int N, int H, int W, int Cin, int Cout,
                 int in_unshuffle, int epi, void* yb, float* yf, const float* r1, const float* r2, const float* r3,
                 const void* aux, float* part, float alpha, int dtype, void* stream) {
  if (dtype != SRMI_DTYPE_BF16 && dtype != SRMI_DTYPE_F32) return SRMI_ERR_ARG;
  ConvParams p{};
  p.f32 = dtype == SRMI_DTYPE_F32;
  p.x = (const bf16_t*)x;
  p.w = (const bf16_t*)wpack;
  p.bias = bias;
  p.N = N;
  p.H = H;
  p.W = W;
  p.Cin = Cin;
  p.Cout = Cout;
  p.in_mode = in_unshuffle ? IN_UNSHUF : IN_PLAIN;
  p.yb = (bf16_t*)yb;
  p.yf = yf;
  p.r1 = r1;
  p.r2 = r2;
  p.r3 = r3;
  p.aux = (const bf16_t*)aux;
  p.part = part;
  p.part_stride = (epi == EPI_DG_ACC || epi == EPI_DG_ACC_CA) ? 128 : Cout;
  p.alpha = alpha;
  return conv3x3_launch(p, epi, S_(stream));
}

int srmi_conv3x3_nstrips(int H, int W) { return conv3x3_nstrips(H, W); }

// diagnostic only: s_memtime stamps of the conv kernel (64 per workgroup), NULL = off
int srmi_debug_conv_stamps(void* buf) {
  conv3x3_set_debug_stamps((unsigned long long*)buf);
  return 0;
}

int srmi_debug_wgrad_stamps(void* buf) {
  wgrad3x3_set_debug_stamps((unsigned long long*)buf);
  return 0;
}

int srmi_pack_conv(const float* w, const float* b, int Cout, int Cin, int ps, void* fpack, void* dpack, float* pbias,
                   int dtype, void* stream) {
  if (dtype != SRMI_DTYPE_BF16 && dtype != SRMI_DTYPE_F32) return SRMI_ERR_ARG;
  return pack_one_launch(w, b, Cout, Cin, ps, fpack, dpack, pbias, dtype == SRMI_DTYPE_F32, S_(stream));
}

int srmi_wgrad3x3(const void* x, const void* dy, int N, int H, int W, int Cout, int dy_unshuffle, int row_splits,
                  float* slab, size_t slab_bytes, int ps, float alpha, float* gw, float* gb, int dtype, void* stream) {
  if (dtype != SRMI_DTYPE_BF16 && dtype != SRMI_DTYPE_F32) return SRMI_ERR_ARG;
  WgradParams p{};
  p.f32 = dtype == SRMI_DTYPE_F32;
  p.x = (const bf16_t*)x;
  p.dy = (const bf16_t*)dy;
  p.N = N;
  p.H = H;
  p.W = W;
  p.Cout = Cout;
  p.dy_mode = dy_unshuffle ? IN_UNSHUF : IN_PLAIN;
  p.imgs_per_wg = 1;
  p.row_splits = row_splits > 0 ? row_splits : choose_row_splits(N, H, Cout);
  const size_t ns = (size_t)wgrad3x3_nslabs(p);
  const size_t need = ns * Cout * 577 * sizeof(float) + 256;
  if (slab_bytes < need) return SRMI_ERR_WORKSPACE;
  p.slab = slab;
  p.bslab = slab + ns * Cout * 576;
  RC(wgrad3x3_launch(p, S_(stream)));
  if (!gw && !gb) return 0;  // partial slabs only (profiling the MFMA kernel alone)
  return wgrad_reduce_launch(p.slab, p.bslab, (int)ns, Cout, ps, wgrad3x3_slab_layout(p), alpha, gw, gb, S_(stream));
}

int srmi_ca_forward(const void* u, const float* part, int nstrips, const float* w1, const float* b1, const float* w2,
                    const float* b2, int N, int HW, int C, int R, const float* h_in, float* h_out, void* hb_out,
                    float* rec, int dtype, void* stream) {
  if (dtype != SRMI_DTYPE_BF16 && dtype != SRMI_DTYPE_F32) return SRMI_ERR_ARG;
  return ca_fwd_launch(u, part, nstrips, w1, b1, w2, b2, N, HW, C, R, h_in, h_out, hb_out, rec,
                       dtype == SRMI_DTYPE_F32, S_(stream));
}

int srmi_ca_forward_pair(const void* u, const float* part, int nstrips, const float* w1, const float* b1,
                         const float* w2, const float* b2, int N, int HW, int C, int R, const float* h_in,
                         const void* hi_in, const void* lo_in, void* hi_out, void* lo_out, float* rec, void* stream) {
  if (!hi_out || !lo_out || (!h_in && (!hi_in || !lo_in))) return SRMI_ERR_ARG;
  return ca_fwd_launch(u, part, nstrips, w1, b1, w2, b2, N, HW, C, R, h_in, nullptr, hi_out, rec, 0, S_(stream),
                       h_in ? nullptr : hi_in, h_in ? nullptr : lo_in, lo_out);
}

int srmi_ca_backward(const float* g, const float* part, int nstrips, const float* rec, const float* w1,
                     const float* w2, int N, int HW, int C, int R, void* du, float* brec, int dtype, void* stream) {
  if (dtype != SRMI_DTYPE_BF16 && dtype != SRMI_DTYPE_F32) return SRMI_ERR_ARG;
  return ca_bwd_du_launch(g, 0, part, nstrips, rec, w1, w2, N, HW, C, R, du, brec, dtype == SRMI_DTYPE_F32,
                          S_(stream));
}

int srmi_head_forward(const float* lr, const float* w, const float* b, int N, int C, int H, int W, float* x0f,
                      void* x0b, int dtype, void* stream) {
  if (dtype != SRMI_DTYPE_BF16 && dtype != SRMI_DTYPE_F32) return SRMI_ERR_ARG;
  return head_fwd_launch(lr, w, b, N, C, H, W, x0f, x0b, dtype == SRMI_DTYPE_F32, S_(stream));
}

int srmi_tail_forward(const void* x, const float* w, const float* b, int N, int C, int H, int W, float* y, int dtype,
                      void* stream) {
  if (dtype != SRMI_DTYPE_BF16 && dtype != SRMI_DTYPE_F32) return SRMI_ERR_ARG;
  return tail_fwd_launch(x, w, b, N, C, H, W, y, dtype == SRMI_DTYPE_F32, S_(stream));
}

int srmi_llc_index_map_workspace(long long n_template, size_t* bytes) {
  if (!bytes) return SRMI_ERR_ARG;
  return llc_index_map_workspace(n_template, bytes);
}

int srmi_llc_index_map(const void* template_be, long long n_template, int nx, int y0, int ys, int x0, int xs,
                       int* idx_map, long long* n_wet, void* workspace, size_t workspace_bytes, void* stream) {
  return llc_index_map_launch(static_cast<const uint32_t*>(template_be), n_template, nx, y0, ys, x0, xs, idx_map,
                              n_wet, workspace, workspace_bytes, S_(stream));
}

int srmi_llc_gather(const void* data_be, long long n_values, const int* idx_map, long long npix, float* out,
                    void* stream) {
  return llc_gather_launch(static_cast<const uint32_t*>(data_be), n_values, idx_map, npix, out, S_(stream));
}

int srmi_tiles_nonfinite(const float* region, int C, int H, int W, int ty, int tx, int* bad, void* stream) {
  return tiles_nonfinite_launch(region, C, H, W, ty, tx, bad, S_(stream));
}

int srmi_tiles_gather(const float* region, int C, int H, int W, int ty, int tx, const int* src, int nslots,
                      float* out, void* stream) {
  return tiles_gather_launch(region, C, H, W, ty, tx, src, nslots, out, S_(stream));
}

int srmi_batch_prep(const float* raw, int B, int C, int T, int flip_index, int scale, float* hr, float* lr,
                    float* mean, float* std, void* stream) {
  return batch_prep_launch(raw, B, C, T, flip_index, scale, hr, lr, mean, std, S_(stream));
}

int srmi_region_to_tiles(const float* region, int C, int H, int W, int ty, int tx, float* tiles, float* mean,
                         float* std, int* bad, void* stream) {
  if (!region || !tiles || !mean || !std) return SRMI_ERR_ARG;
  return region_to_tiles_launch(region, C, H, W, ty, tx, tiles, mean, std, bad, S_(stream));
}

int srmi_tiles_to_region(const float* tiles, const float* mean, const float* std, const int* inv, int C, int ty,
                         int tx, int gy, int gx, float* out, void* stream) {
  if (!tiles || !out || (mean && !std)) return SRMI_ERR_ARG;
  return tiles_to_region_launch(tiles, mean, std, inv, C, ty, tx, gy, gx, out, S_(stream));
}

int srmi_axpy(float* y, const float* x, float a, size_t n, void* stream) {
  if (!y || !x) return SRMI_ERR_ARG;
  return scale_add_launch(y, x, a, n, S_(stream));
}

}  // extern "C"
