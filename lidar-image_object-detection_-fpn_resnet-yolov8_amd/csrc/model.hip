// FPN-ResNet-18 (KFPN) model: reference state_dict layout, host-side weight
// packing (BatchNorm folding + OHWI re-layout) and the forward orchestration.
//
// Reference: models/fpn_resnet.py:112-301 (PoseResNet, BasicBlock, get_pose_net),
//            models/model_utils.py:25-43 (create_model).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "aux_kernels.h"
#include "conv.h"

namespace sfa {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}

struct Entry {
  std::string name;
  std::vector<int64_t> shape;
};

static int64_t numel(const Entry& e) {
  int64_t n = 1;
  for (auto s : e.shape) n *= s;
  return n;
}

static const int kFpnC[3] = {256, 128, 64};

static int check_arch(const sfa_arch* a) {
  SFA_CHECK_ARG(a != nullptr, "arch is null");
  if (a->num_layers != 18) {
    set_error("only fpn_resnet_18 is implemented (got %d layers)", a->num_layers);
    return SFA_E_UNSUPPORTED;
  }
  if (a->head_conv != 64) {
    set_error("only head_conv = 64 is implemented (got %d)", a->head_conv);
    return SFA_E_UNSUPPORTED;
  }
  SFA_CHECK_ARG(a->num_heads >= 1 && a->num_heads <= SFA_MAX_HEADS, "num_heads %d out of range",
                a->num_heads);
  for (int j = 0; j < a->num_heads; ++j) {
    SFA_CHECK_ARG(a->head_channels[j] >= 1 && a->head_channels[j] <= 4,
                  "head %d: channels %d out of [1, 4]", j, a->head_channels[j]);
    SFA_CHECK_ARG(strnlen(a->head_names[j], 32) > 0 && strnlen(a->head_names[j], 32) < 32,
                  "head %d: bad name", j);
  }
  return SFA_OK;
}

static std::vector<int> sorted_heads(const sfa_arch* a) {
  std::vector<int> idx(a->num_heads);
  for (int j = 0; j < a->num_heads; ++j) idx[j] = j;
  std::sort(idx.begin(), idx.end(), [&](int x, int y) {
    return std::string(a->head_names[x]) < std::string(a->head_names[y]);
  });
  return idx;
}

// nn.Module registration order of PoseResNet (fpn_resnet.py:114-151, 42-53).
static std::vector<Entry> state_layout(const sfa_arch* a) {
  std::vector<Entry> v;
  auto bn = [&](const std::string& p, int64_t c) {
    v.push_back({p + ".weight", {c}});
    v.push_back({p + ".bias", {c}});
    v.push_back({p + ".running_mean", {c}});
    v.push_back({p + ".running_var", {c}});
    v.push_back({p + ".num_batches_tracked", {}});
  };
  v.push_back({"conv1.weight", {64, 3, 7, 7}});
  bn("bn1", 64);
  int inplanes = 64;
  for (int li = 1; li <= 4; ++li) {
    const int planes = 64 << (li - 1);
    for (int bi = 0; bi < 2; ++bi) {
      const std::string p = "layer" + std::to_string(li) + "." + std::to_string(bi);
      const int cin = bi == 0 ? inplanes : planes;
      v.push_back({p + ".conv1.weight", {planes, cin, 3, 3}});
      bn(p + ".bn1", planes);
      v.push_back({p + ".conv2.weight", {planes, planes, 3, 3}});
      bn(p + ".bn2", planes);
      if (bi == 0 && (li > 1)) {
        v.push_back({p + ".downsample.0.weight", {planes, inplanes, 1, 1}});
        bn(p + ".downsample.1", planes);
      }
    }
    inplanes = planes;
  }
  const int up_out[3] = {256, 128, 64}, up_in[3] = {768, 384, 192};
  for (int i = 0; i < 3; ++i) {
    const std::string p = "conv_up_level" + std::to_string(i + 1);
    v.push_back({p + ".weight", {up_out[i], up_in[i], 1, 1}});
    v.push_back({p + ".bias", {up_out[i]}});
  }
  const auto order = sorted_heads(a);
  for (int f = 0; f < 3; ++f)
    for (int j : order) {
      const std::string p = "fpn" + std::to_string(f) + "_" + a->head_names[j];
      v.push_back({p + ".0.weight", {a->head_conv, kFpnC[f], 3, 3}});
      v.push_back({p + ".0.bias", {a->head_conv}});
      v.push_back({p + ".2.weight", {a->head_channels[j], a->head_conv, 1, 1}});
      v.push_back({p + ".2.bias", {a->head_channels[j]}});
    }
  return v;
}

// ----------------------------------------------------------- packed layout
// Offsets in floats into the packed buffer.  wx: the same weights split into three
// bf16 terms [3][N][Kpad] for the bf16x6 kernels (conv_x6_kernel.h); wh / winv: the
// fp16x3 form, W[n][k] * 2^e[n] as two fp16 terms [2][N][Kpad] and winv[n] = 2^-e[n].
struct PConv {
  size_t w, b, wx, wh, winv;
  int N, K, Kpad;
};
struct PHeads {
  size_t w3, b3, w1, b1, wx, wh, winv;
  int N, K;
};
struct Plan {
  PConv stem;
  PConv blk[4][2][2];  // [layer][block][conv1, conv2(+downsample)]
  PConv fpn[3];
  PHeads heads[3];
  size_t total;
};

static Plan make_plan(const sfa_arch* a) {
  Plan p;
  size_t cur = 0;
  auto take = [&](size_t n) {
    const size_t o = cur;
    cur = align_up(cur + n, 16);
    return o;
  };
  auto conv = [&](int N, int K) {
    PConv c;
    c.N = N;
    c.K = K;
    c.Kpad = (int)align_up(K, 16);
    c.w = take((size_t)N * c.Kpad);
    c.b = take(N);
    c.wx = take(((size_t)3 * N * c.Kpad + 1) / 2);
    c.wh = take((size_t)N * c.Kpad);
    c.winv = take(N);
    return c;
  };
  p.stem = conv(64, 49 * 4);
  int inplanes = 64;
  for (int li = 0; li < 4; ++li) {
    const int planes = 64 << li;
    for (int bi = 0; bi < 2; ++bi) {
      const int cin = bi == 0 ? inplanes : planes;
      const bool ds = bi == 0 && li > 0;
      p.blk[li][bi][0] = conv(planes, 9 * cin);
      p.blk[li][bi][1] = conv(planes, 9 * planes + (ds ? inplanes : 0));
    }
    inplanes = planes;
  }
  p.fpn[0] = conv(256, 768);
  p.fpn[1] = conv(128, 384);
  p.fpn[2] = conv(64, 192);
  for (int f = 0; f < 3; ++f) {
    PHeads& h = p.heads[f];
    h.N = a->num_heads * a->head_conv;
    h.K = 9 * kFpnC[f];
    h.w3 = take((size_t)h.N * h.K);
    h.b3 = take(h.N);
    h.w1 = take((size_t)a->num_heads * 4 * 64);
    h.b1 = take((size_t)a->num_heads * 4);
    h.wx = take(((size_t)3 * h.N * h.K + 1) / 2);
    h.wh = take((size_t)h.N * h.K);
    h.winv = take(h.N);
  }
  p.total = cur;
  return p;
}

struct StateView {
  std::map<std::string, std::pair<const float*, Entry>> m;
  const float* get(const std::string& n) const {
    auto it = m.find(n);
    return it == m.end() ? nullptr : it->second.first;
  }
};

// OIHW conv weight folded by BN scale into W[o][(kh*KW+kw)*Cpad + c] + k_off.
static void put_conv(float* W, int Kpad, int k_off, const float* w, int O, int I, int KH, int KW,
                     int Cpad, const std::vector<double>& scale) {
  for (int o = 0; o < O; ++o)
    for (int c = 0; c < I; ++c)
      for (int kh = 0; kh < KH; ++kh)
        for (int kw = 0; kw < KW; ++kw) {
          const double v = w[((o * I + c) * KH + kh) * KW + kw];
          W[(size_t)o * Kpad + k_off + (kh * KW + kw) * Cpad + c] = (float)(v * scale[o]);
        }
}

static void bn_fold(const StateView& s, const std::string& p, int C, std::vector<double>& scale,
                    std::vector<double>& shift) {
  const float* g = s.get(p + ".weight");
  const float* b = s.get(p + ".bias");
  const float* mu = s.get(p + ".running_mean");
  const float* var = s.get(p + ".running_var");
  scale.assign(C, 1.0);
  shift.assign(C, 0.0);
  for (int c = 0; c < C; ++c) {
    scale[c] = (double)g[c] / std::sqrt((double)var[c] + 1e-5);
    shift[c] = (double)b[c] - (double)mu[c] * scale[c];
  }
}

// f32 -> bf16, round to nearest even (finite inputs)
static uint16_t bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// W (n floats) -> three bf16 terms t0 + t1 + t2 == W (each residual is exact in f32)
static void split_terms(const float* w, size_t n, uint16_t* out) {
  for (size_t i = 0; i < n; ++i) {
    float x = w[i];
    for (int t = 0; t < 3; ++t) {
      const uint16_t b = bf16_rne(x);
      out[t * n + i] = b;
      uint32_t u = (uint32_t)b << 16;
      float bf;
      memcpy(&bf, &u, 4);
      x -= bf;
    }
  }
}

// fp16x3 form of W [N][K]: per output channel n, e[n] = floor(log2 max_k |W[n][k]|) and
// W * 2^(13 - e[n]) (every |.| < 2^14) = hi + lo with hi = fp16(.) and lo = fp16(. - hi);
// winv[n] = 2^(e[n] - 13).  Zero rows keep scale 1.
static void split_terms_h3(const float* w, int N, int K, uint16_t* out, float* winv) {
  const size_t n = (size_t)N * K;
  for (int o = 0; o < N; ++o) {
    float mx = 0.f;
    for (int k = 0; k < K; ++k) mx = std::max(mx, std::fabs(w[(size_t)o * K + k]));
    int e = 13;
    if (mx > 0.f) {
      (void)std::frexp(mx, &e);  // mx in [2^(e-1), 2^e)
      e -= 1;
    }
    const float sc = std::ldexp(1.f, 13 - e);
    winv[o] = std::ldexp(1.f, e - 13);
    for (int k = 0; k < K; ++k) {
      const size_t i = (size_t)o * K + k;
      const float x = w[i] * sc;
      const _Float16 hi = (_Float16)x;
      const _Float16 lo = (_Float16)(x - (float)hi);
      memcpy(out + i, &hi, 2);
      memcpy(out + n + i, &lo, 2);
    }
  }
}

}  // namespace sfa

using namespace sfa;

struct sfa_model {
  sfa_arch arch;
  const float* w;
  Plan plan;
  int math;
  int fpn_commute = 7;  // fp16x3: bit f -> FPN conv f as up(W_a x) + W_b skip (env SFA_FPN_COMMUTE, mask)
  // fp16x3 stem form (env SFA_STEM_PATCH): 1 (default) = the 16 x 16 patch kernel + its merge pass
  // (stem_patch_kernel.h); 0 = the implicit-GEMM stem conv + the max-pool kernel, as the other math
  // modes (the round-4 full-width band stem measured slower: tools/experiments/r04)
  int stem_patch = 1;
  // fp16x3 FPN 1x1 convs on the persistent kernels of fpn_kernel.h, mask (env SFA_FPN_GEMM): bit f =
  // level f's low-resolution W_a . x conv (weight-resident row streaming), bit 3 + f = its skip conv
  // with the upsampled residual (level 2: full rows with the taps from an LDS ring; levels 0 / 1: flat
  // pixel steps, fpn_seg_kernel); the other convs run on conv_h3 / conv_r3 (the same products for the
  // skip convs). Default 61 = the low-res convs of levels 0 and 2 and the three skip convs, the ones
  // measured faster (profiles/r04d_*, r04l_*, r05n_*); 63 (level 1's low-res conv too: -5 us serial, other
  // bits within 2e-5) measured bench-equal
  int fpn_gemm = 61;
  // fp16x3 split-K layer4 strip convs: 1 (default) = the last slice of each tile combines the partials in
  // the conv kernel (tickets, conv_h3_kernel.h splitk_ticket), 0 = splitk_reduce_kernel launches; the
  // same bits (env SFA_SPLITK_TICKETS). conv_h3's split convs keep the reduce launch.
  int splitk_tickets = 1;
  // Side stream for the level-0 heads (they only need up_level2, so they overlap the rest
  // of the FPN and the level-1/2 heads); created with the model on the current device,
  // used only when the forward's stream is on that device.
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr, mid = nullptr;
  int device = -1;
  std::mutex fork_mu;  // fork ... join of one forward is not interleaved with another's
  // Kernel probe (sfa_model_set_probe): timing events around each head-level launch, recorded
  // on the stream that launches it (never while that stream is being captured); PROBE_SERIAL
  // keeps every launch on the caller's stream so each head launch has the chip to itself.
  int probe = 0;
  hipEvent_t probe_ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
};

// The model's side stream(s) and their events, created on the current device; on failure
// (no device) none, and the forward runs every launch on the caller's stream.
static void drop_side_streams(sfa_model* m) {
  for (hipEvent_t* e : {&m->fork, &m->join, &m->mid})
    if (*e) {
      (void)hipEventDestroy(*e);
      *e = nullptr;
    }
  if (m->side) {
    (void)hipStreamDestroy(m->side);
    m->side = nullptr;
  }
}

static void make_side_streams(sfa_model* m) {
  if (hipGetDevice(&m->device) != hipSuccess || hipStreamCreateWithFlags(&m->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&m->fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&m->join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&m->mid, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    drop_side_streams(m);
  }
}

extern "C" int sfa_abi_version(void) { return SFA_ABI_VERSION; }
extern "C" const char* sfa_last_error_string(void) { return g_err.c_str(); }

extern "C" int sfa_state_count(const sfa_arch* arch) {
  if (check_arch(arch) != SFA_OK) return -1;
  return (int)state_layout(arch).size();
}

extern "C" int sfa_state_entry(const sfa_arch* arch, int index, char* name, int name_len,
                               int64_t* shape4, int* ndim) {
  int rc = check_arch(arch);
  if (rc != SFA_OK) return rc;
  const auto v = state_layout(arch);
  SFA_CHECK_ARG(index >= 0 && index < (int)v.size(), "state index %d out of range", index);
  const Entry& e = v[index];
  SFA_CHECK_ARG(name && name_len > (int)e.name.size(), "name buffer too small");
  memcpy(name, e.name.c_str(), e.name.size() + 1);
  for (int i = 0; i < 4; ++i) shape4[i] = i < (int)e.shape.size() ? e.shape[i] : 0;
  *ndim = (int)e.shape.size();
  return SFA_OK;
}

extern "C" size_t sfa_state_floats(const sfa_arch* arch) {
  if (check_arch(arch) != SFA_OK) return 0;
  size_t n = 0;
  for (const auto& e : state_layout(arch))
    if (e.name.find("num_batches_tracked") == std::string::npos) n += numel(e);
  return n;
}

extern "C" size_t sfa_packed_floats(const sfa_arch* arch) {
  if (check_arch(arch) != SFA_OK) return 0;
  return make_plan(arch).total;
}

extern "C" int sfa_pack_weights(const sfa_arch* arch, const float* state, size_t state_floats,
                                float* packed) {
  int rc = check_arch(arch);
  if (rc != SFA_OK) return rc;
  SFA_CHECK_ARG(state && packed, "pack: null argument");
  SFA_CHECK_ARG(state_floats == sfa_state_floats(arch), "pack: expected %zu state floats, got %zu",
                sfa_state_floats(arch), state_floats);
  StateView s;
  size_t off = 0;
  for (const auto& e : state_layout(arch)) {
    if (e.name.find("num_batches_tracked") != std::string::npos) continue;
    s.m[e.name] = {state + off, e};
    off += numel(e);
  }
  const Plan p = make_plan(arch);
  std::fill(packed, packed + p.total, 0.f);
  std::vector<double> sc, sh, sc2, sh2;

  // stem: conv1 + bn1, input channels padded 3 -> 4
  bn_fold(s, "bn1", 64, sc, sh);
  put_conv(packed + p.stem.w, p.stem.Kpad, 0, s.get("conv1.weight"), 64, 3, 7, 7, 4, sc);
  for (int o = 0; o < 64; ++o) packed[p.stem.b + o] = (float)sh[o];

  int inplanes = 64;
  for (int li = 0; li < 4; ++li) {
    const int planes = 64 << li;
    for (int bi = 0; bi < 2; ++bi) {
      const std::string pre = "layer" + std::to_string(li + 1) + "." + std::to_string(bi);
      const int cin = bi == 0 ? inplanes : planes;
      const PConv& c1 = p.blk[li][bi][0];
      bn_fold(s, pre + ".bn1", planes, sc, sh);
      put_conv(packed + c1.w, c1.Kpad, 0, s.get(pre + ".conv1.weight"), planes, cin, 3, 3, cin, sc);
      for (int o = 0; o < planes; ++o) packed[c1.b + o] = (float)sh[o];
      const PConv& c2 = p.blk[li][bi][1];
      bn_fold(s, pre + ".bn2", planes, sc, sh);
      put_conv(packed + c2.w, c2.Kpad, 0, s.get(pre + ".conv2.weight"), planes, planes, 3, 3, planes,
               sc);
      if (bi == 0 && li > 0) {
        bn_fold(s, pre + ".downsample.1", planes, sc2, sh2);
        put_conv(packed + c2.w, c2.Kpad, 9 * planes, s.get(pre + ".downsample.0.weight"), planes,
                 inplanes, 1, 1, inplanes, sc2);
        for (int o = 0; o < planes; ++o) packed[c2.b + o] = (float)(sh[o] + sh2[o]);
      } else {
        for (int o = 0; o < planes; ++o) packed[c2.b + o] = (float)sh[o];
      }
    }
    inplanes = planes;
  }
  const int up_out[3] = {256, 128, 64}, up_in[3] = {768, 384, 192};
  for (int i = 0; i < 3; ++i) {
    const std::string pre = "conv_up_level" + std::to_string(i + 1);
    std::vector<double> one(up_out[i], 1.0);
    put_conv(packed + p.fpn[i].w, p.fpn[i].Kpad, 0, s.get(pre + ".weight"), up_out[i], up_in[i], 1,
             1, up_in[i], one);
    const float* b = s.get(pre + ".bias");
    for (int o = 0; o < up_out[i]; ++o) packed[p.fpn[i].b + o] = b[o];
  }
  for (int f = 0; f < 3; ++f) {
    const PHeads& hp = p.heads[f];
    std::vector<double> one(arch->head_conv, 1.0);
    for (int j = 0; j < arch->num_heads; ++j) {
      const std::string pre = "fpn" + std::to_string(f) + "_" + arch->head_names[j];
      put_conv(packed + hp.w3 + (size_t)j * 64 * hp.K, hp.K, 0, s.get(pre + ".0.weight"), 64,
               kFpnC[f], 3, 3, kFpnC[f], one);
      const float* b3 = s.get(pre + ".0.bias");
      for (int o = 0; o < 64; ++o) packed[hp.b3 + j * 64 + o] = b3[o];
      const float* w1 = s.get(pre + ".2.weight");
      const float* b1 = s.get(pre + ".2.bias");
      for (int c = 0; c < arch->head_channels[j]; ++c) {
        for (int k = 0; k < 64; ++k) packed[hp.w1 + (j * 4 + c) * 64 + k] = w1[c * 64 + k];
        packed[hp.b1 + j * 4 + c] = b1[c];
      }
    }
  }
  // bf16x6 and fp16x3 terms of every implicit-GEMM weight matrix
  auto split = [&](const PConv& c) {
    split_terms(packed + c.w, (size_t)c.N * c.Kpad, reinterpret_cast<uint16_t*>(packed + c.wx));
    split_terms_h3(packed + c.w, c.N, c.Kpad, reinterpret_cast<uint16_t*>(packed + c.wh),
                   packed + c.winv);
  };
  split(p.stem);
  for (int li = 0; li < 4; ++li)
    for (int bi = 0; bi < 2; ++bi)
      for (int ci = 0; ci < 2; ++ci) split(p.blk[li][bi][ci]);
  for (int i = 0; i < 3; ++i) split(p.fpn[i]);
  for (int f = 0; f < 3; ++f) {
    const PHeads& hp = p.heads[f];
    split_terms(packed + hp.w3, (size_t)hp.N * hp.K, reinterpret_cast<uint16_t*>(packed + hp.wx));
    split_terms_h3(packed + hp.w3, hp.N, hp.K, reinterpret_cast<uint16_t*>(packed + hp.wh),
                   packed + hp.winv);
  }
  return SFA_OK;
}

extern "C" int sfa_model_create(const sfa_arch* arch, const float* packed_device, sfa_model** out) {
  int rc = check_arch(arch);
  if (rc != SFA_OK) return rc;
  SFA_CHECK_ARG(packed_device && out, "model_create: null argument");
  sfa_model* m = new sfa_model;
  m->arch = *arch;
  m->w = packed_device;
  m->plan = make_plan(arch);
  m->math = SFA_MATH_FP16X3;
  // A/B convenience: the environment seeds the options once, here (sfa_model_set_option
  // overrides them; nothing reads the environment on the launch path)
  if (const char* e = getenv("SFA_STEM_PATCH")) m->stem_patch = atoi(e) != 0;
  if (const char* e = getenv("SFA_FPN_COMMUTE")) m->fpn_commute = atoi(e) & 7;
  if (const char* e = getenv("SFA_FPN_GEMM")) m->fpn_gemm = atoi(e) & 63;
  if (const char* e = getenv("SFA_SPLITK_TICKETS")) m->splitk_tickets = atoi(e) != 0;
  bool side_streams = true;  // env SFA_SIDE_STREAMS=0: every launch on the caller's stream (A/B)
  if (const char* e = getenv("SFA_SIDE_STREAMS")) side_streams = strcmp(e, "0") != 0;
  if (side_streams) make_side_streams(m);
  *out = m;
  return SFA_OK;
}

extern "C" void sfa_model_destroy(sfa_model* model) {
  if (!model) return;
  for (hipEvent_t e : model->probe_ev)
    if (e) (void)hipEventDestroy(e);
  drop_side_streams(model);
  delete model;
}

extern "C" int sfa_model_set_side_streams(sfa_model* model, int on) {
  SFA_CHECK_ARG(model, "set_side_streams: null model");
  std::lock_guard<std::mutex> lk(model->fork_mu);
  if (!on && model->side) {
    // the side streams' last forward must be done before they go (the caller's stream has
    // joined them, so nothing enqueued later depends on them)
    SFA_HIP_TRY(hipStreamSynchronize(model->side));
    drop_side_streams(model);
  } else if (on && !model->side) {
    make_side_streams(model);
    SFA_CHECK_ARG(model->side, "set_side_streams: no side stream could be created on this device");
  }
  return SFA_OK;
}

extern "C" int sfa_model_set_option(sfa_model* model, int key, int value) {
  SFA_CHECK_ARG(model, "set_option: null model");
  std::lock_guard<std::mutex> lk(model->fork_mu);
  switch (key) {
    case SFA_OPT_STEM_PATCH:
      SFA_CHECK_ARG(value == 0 || value == 1, "set_option: STEM_PATCH %d not 0 / 1", value);
      model->stem_patch = value;
      break;
    case SFA_OPT_FPN_COMMUTE:
      SFA_CHECK_ARG(value >= 0 && value <= 7, "set_option: FPN_COMMUTE mask %d not in 0..7", value);
      model->fpn_commute = value;
      break;
    case SFA_OPT_FPN_GEMM:
      SFA_CHECK_ARG(value >= 0 && value <= 63, "set_option: FPN_GEMM mask %d not in 0..63", value);
      model->fpn_gemm = value;
      break;
    case SFA_OPT_SPLITK_TICKETS:
      SFA_CHECK_ARG(value == 0 || value == 1, "set_option: SPLITK_TICKETS %d not 0 / 1", value);
      model->splitk_tickets = value;
      break;
    default: set_error("set_option: unknown key %d", key); return SFA_E_INVALID;
  }
  return SFA_OK;
}

extern "C" int sfa_model_get_option(const sfa_model* model, int key, int* value) {
  SFA_CHECK_ARG(model && value, "get_option: null argument");
  switch (key) {
    case SFA_OPT_STEM_PATCH: *value = model->stem_patch; break;
    case SFA_OPT_FPN_COMMUTE: *value = model->fpn_commute; break;
    case SFA_OPT_FPN_GEMM: *value = model->fpn_gemm; break;
    case SFA_OPT_SPLITK_TICKETS: *value = model->splitk_tickets; break;
    default: set_error("get_option: unknown key %d", key); return SFA_E_INVALID;
  }
  return SFA_OK;
}

extern "C" int sfa_model_set_math(sfa_model* model, int math) {
  SFA_CHECK_ARG(model, "set_math: null model");
  SFA_CHECK_ARG(math == SFA_MATH_F32 || math == SFA_MATH_BF16X6 || math == SFA_MATH_FP16X3,
                "set_math: unknown mode %d", math);
  model->math = math;
  return SFA_OK;
}

extern "C" int sfa_model_get_math(const sfa_model* model) { return model ? model->math : -1; }

extern "C" int sfa_model_set_probe(sfa_model* model, int flags) {
  SFA_CHECK_ARG(model, "set_probe: null model");
  SFA_CHECK_ARG((flags & ~(SFA_PROBE_HEADS | SFA_PROBE_SERIAL)) == 0, "set_probe: unknown flags %d", flags);
  if (flags & SFA_PROBE_HEADS)
    for (hipEvent_t& e : model->probe_ev)
      if (!e) SFA_HIP_TRY(hipEventCreate(&e));
  model->probe = flags;
  return SFA_OK;
}

extern "C" int sfa_model_probe_times(const sfa_model* model, float* ms, int n) {
  SFA_CHECK_ARG(model && ms && n >= 0 && n <= 3, "probe_times: bad arguments");
  SFA_CHECK_ARG(model->probe & SFA_PROBE_HEADS, "probe_times: probe not enabled");
  for (int f = 0; f < n; ++f) {
    SFA_HIP_TRY(hipEventSynchronize(model->probe_ev[2 * f + 1]));
    SFA_HIP_TRY(hipEventElapsedTime(&ms[f], model->probe_ev[2 * f], model->probe_ev[2 * f + 1]));
  }
  return SFA_OK;
}

namespace sfa {

// Activation buffers of one forward (NHWC f32), carved from the workspace.
struct Bufs {
  size_t xin, s0, p0, t[4], a[4], l[4], up1, c1, up2, c2, up3, up4, L0, L1, L2, amax, tick, tick_words, part,
      part_floats, total;
};

// fp16x3 activation maxima (conv.h): per tensor a conv reads (named by its producer), B
// frames of SFA_AMAX_WORDS words.  Pooling and bilinear upsampling never raise max |x|, so their
// outputs share their input's slot.
enum AmaxSlot { AM_INPUT = 0, AM_STEM = 1, AM_BLK = 2 /* + 4 li + 2 bi + ci */, AM_FPN = 18,
                AM_COUNT = 21 };

static Bufs plan_bufs(const sfa_arch* arch, int B, int H, int W) {
  Bufs b;
  size_t cur = 0;
  auto take = [&](size_t floats) {
    const size_t o = cur;
    cur = align_up(cur + floats * 4, 256);
    return o;
  };
  const size_t P2 = (size_t)(H / 2) * (W / 2), P4 = (size_t)(H / 4) * (W / 4);
  b.xin = take((size_t)B * H * W * 4);
  b.s0 = take((size_t)B * P2 * 64);
  b.p0 = take((size_t)B * P4 * 64);
  for (int li = 0; li < 4; ++li) {
    const size_t px = (size_t)(H >> (li + 2)) * (W >> (li + 2));
    const size_t n = (size_t)B * px * (64 << li);
    b.t[li] = take(n);
    b.a[li] = take(n);
    b.l[li] = take(n);
  }
  const size_t P8 = (size_t)(H / 8) * (W / 8), P16 = (size_t)(H / 16) * (W / 16);
  b.up1 = take((size_t)B * P16 * 512);
  b.c1 = take((size_t)B * P16 * 256);
  b.up2 = take((size_t)B * P8 * 256);
  b.c2 = take((size_t)B * P8 * 128);
  b.up3 = take((size_t)B * P4 * 128);
  b.up4 = take((size_t)B * P4 * 64);
  int nch = 0;
  for (int j = 0; j < arch->num_heads; ++j) nch += arch->head_channels[j];
  b.L0 = take((size_t)nch * B * P8);
  b.L1 = take((size_t)nch * B * P4);
  b.L2 = take((size_t)nch * B * P4);
  // the activation maxima and the split-K tickets (one zeroing memset per forward, right after them)
  b.amax = take((size_t)AM_COUNT * B * SFA_AMAX_WORDS);
  // split-K tickets (conv_h3_kernel.h splitk_ticket): one word per output tile of each of the four
  // layer4 convs, for tiles of >= 64 x 64
  b.tick_words = (size_t)((B * (H / 32) * (W / 32) + 63) / 64) * (512 / 64);
  b.tick = take(4 * b.tick_words);
  // split-K partial sums (conv.hip pick_ksplit: 2 slices of the 512-wide layer4 convs)
  b.part_floats = (size_t)2 * B * (H / 32) * (W / 32) * 512;
  b.part = take(b.part_floats);
  b.total = cur;
  return b;
}

static ConvSeg seg(const float* x, int B, int H, int W, int C, int k, int stride, int pad) {
  ConvSeg g;
  make_seg(g, x, B, H, W, C, k, stride, pad);  // oversize inputs are rejected by launch_conv
  return g;
}

static ConvArgs conv_args(const float* wbase, const PConv& pc, int B, int OH, int OW, float* y,
                          const float* res, int relu) {
  ConvArgs a;
  memset(&a, 0, sizeof a);
  a.nseg = 1;
  a.Kpad = pc.Kpad;
  a.w = wbase + pc.w;
  a.wx = reinterpret_cast<const uint16_t*>(wbase + pc.wx);
  a.wh = reinterpret_cast<const uint16_t*>(wbase + pc.wh);
  a.winv = wbase + pc.winv;
  a.bias = wbase + pc.b;
  a.res = res;
  a.y = y;
  a.M = B * OH * OW;
  a.N = pc.N;
  a.OH = OH;
  a.OW = OW;
  a.relu = relu;
  return a;
}

}  // namespace sfa

// Frames one forward pass runs at once (sfa_forward_max_batch): every conv kernel reads its input
// segments through buffer resources with 32-bit byte offsets (conv.hip launch_conv: < 2 GiB). The
// widest conv input per frame is up_level3 / the level-1 heads' input, (H/4)(W/4) x 128 floats =
// 32 H W bytes (the stem input, 12-16 H W bytes, and every other map are smaller), so a pass holds
// floor((2^31 - 1) / (32 H W)) frames: 181 at 608 x 608. Larger batches run in passes of that
// many frames (sfa_model_forward); frames are independent and their arithmetic batch-invariant
// (per-frame fp16x3 scales), so the chunking changes no bit.
static int forward_max_batch(int H, int W) {
  if (H <= 0 || W <= 0) return 0;
  const unsigned long long per_frame = 32ull * (unsigned long long)H * (unsigned long long)W;
  const unsigned long long n = ((1ull << 31) - 1) / per_frame;
  return n > 0x7fffffffull ? 0x7fffffff : (int)n;
}

extern "C" int sfa_forward_max_batch(int height, int width) { return forward_max_batch(height, width); }

extern "C" size_t sfa_forward_workspace_size(const sfa_model* m, int batch, int height, int width) {
  if (!m || batch <= 0 || height <= 0 || width <= 0) return 0;
  const int bmax = forward_max_batch(height, width);
  if (bmax < 1) return 0;
  return plan_bufs(&m->arch, std::min(batch, bmax), height, width).total;
}

extern "C" int64_t sfa_forward_buffer_offset(const sfa_model* m, int batch, int height, int width,
                                             int which) {
  if (!m || batch <= 0 || height <= 0 || width <= 0) return -1;
  const int bmax = forward_max_batch(height, width);
  if (bmax < 1) return -1;
  const Bufs b = plan_bufs(&m->arch, std::min(batch, bmax), height, width);
  switch (which) {
    case SFA_BUF_LAYER1: return (int64_t)b.l[0];
    case SFA_BUF_LAYER2: return (int64_t)b.l[1];
    case SFA_BUF_LAYER3: return (int64_t)b.l[2];
    case SFA_BUF_LAYER4: return (int64_t)b.l[3];
    case SFA_BUF_UP_LEVEL2: return (int64_t)b.up2;
    case SFA_BUF_UP_LEVEL3: return (int64_t)b.up3;
    case SFA_BUF_UP_LEVEL4: return (int64_t)b.up4;
    case SFA_BUF_HEADS_L0: return (int64_t)b.L0;
    case SFA_BUF_HEADS_L1: return (int64_t)b.L1;
    case SFA_BUF_HEADS_L2: return (int64_t)b.L2;
    default: return -1;
  }
}

#define SFA_RC(expr)            \
  do {                          \
    int rc_ = (expr);           \
    if (rc_ != SFA_OK) return rc_; \
  } while (0)

// One pass over B <= forward_max_batch(H, W) frames (arguments checked by sfa_model_forward).
static int forward_pass(const sfa_model* m, const float* x, int in_layout, int B, int H, int W,
                        float* const* head_out, void* workspace, void* stream) {
  const Bufs bf = plan_bufs(&m->arch, B, H, W);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  auto F = [&](size_t off) { return reinterpret_cast<float*>(ws + off); };
  const float* wb = m->w;
  const Plan& p = m->plan;

  // fp16x3: every conv input's max |x| is recorded by its producer (slots zeroed here)
  const bool h3 = m->math == SFA_MATH_FP16X3;
  auto AM = [&](int slot) -> unsigned* {
    return h3 ? reinterpret_cast<unsigned*>(ws + bf.amax) + (size_t)slot * B * SFA_AMAX_WORDS : nullptr;
  };
  auto blk_slot = [](int li, int bi, int ci) { return AM_BLK + 4 * li + 2 * bi + ci; };
  if (h3)  // the amax words and the split-K tickets after them
    SFA_RC(launch_zero_words(ws + bf.amax, bf.tick + 4 * bf.tick_words * 4 - bf.amax, st));
  auto io = [&](ConvArgs& a, int in0, int in1, int out) {
    a.amax_in[0] = in0 >= 0 ? AM(in0) : nullptr;
    a.amax_in[1] = in1 >= 0 ? AM(in1) : nullptr;
    a.amax_out = out >= 0 ? AM(out) : nullptr;
    a.part = F(bf.part);
    a.part_floats = bf.part_floats;
  };

  const int H2 = H / 2, W2 = W / 2;
  // The patch stem (fp16x3) reads the caller's layout itself, scales every tile by its own max |x|
  // and max-pools in its epilogue: no layout conversion, no input amax pass, no max-pool launch
  // (stem_patch_kernel.h).
  const bool patch_stem = h3 && m->stem_patch && H2 % 16 == 0 && W2 % 16 == 0;
  const float* xin = x;
  if (patch_stem) {
  } else if (in_layout != SFA_IN_NHWC4) {
    SFA_RC(launch_nchw3_to_nhwc4(x, F(bf.xin), B, H, W, in_layout == SFA_IN_NCHW3_FLIP_HW,
                                 AM(AM_INPUT), st));
    xin = F(bf.xin);
  } else if (h3) {
    SFA_RC(launch_amax_nhwc4(x, B, H, W, AM(AM_INPUT), st));
  }
  // stem conv7x7/s2/p3 + BN + ReLU (fpn_resnet.py:179-181) + max-pool (:182): the patch stem sends
  // the tile-border cells' parts through a side buffer and a merge pass; otherwise the conv and the
  // max-pool kernel.
  {
    ConvArgs a = conv_args(wb, p.stem, B, H2, W2, patch_stem ? F(bf.p0) : F(bf.s0), nullptr, 1);
    a.seg[0] = seg(xin, B, H, W, 4, 7, 2, 3);  // the patch stem reads NCHW3 planes through it too
    io(a, AM_INPUT, -1, AM_STEM);
    if (patch_stem) {
      a.amax_in[0] = nullptr;  // per-tile scales
      a.stem_in = in_layout == SFA_IN_NHWC4 ? STEM_IN_NHWC4
                                             : (in_layout == SFA_IN_NCHW3_FLIP_HW ? STEM_IN_NCHW3_FLIP : STEM_IN_NCHW3);
      a.part = F(bf.s0);  // the (here unused) unfused stem buffer
      a.part_floats = (size_t)B * H2 * W2 * 64;
      SFA_RC(launch_stem_patch(a, st));
    } else {
      SFA_RC(launch_conv(a, EPI_STD, m->math, st));
    }
  }
  if (!patch_stem) SFA_RC(launch_maxpool3s2(F(bf.s0), F(bf.p0), B, H2, W2, 64, st));  // :182
  // residual layers (fpn_resnet.py:184-187)
  const float* xcur = F(bf.p0);
  int xslot = AM_STEM;  // maxpool keeps the stem's max
  int h = H / 4, w = W / 4, cin = 64;
  // split-K tickets of the layer4 convs (the only split ones, conv.hip pick_ksplit): the slice that
  // finishes last combines the partials in the conv kernel (no reduce launch); fp16x3 only
  auto TK = [&](int li, int ci) -> unsigned* {
    return h3 && li == 3 && m->splitk_tickets ? reinterpret_cast<unsigned*>(ws + bf.tick) + (size_t)ci * bf.tick_words : nullptr;
  };
  for (int li = 0; li < 4; ++li) {
    const int planes = 64 << li;
    const int stride = li == 0 ? 1 : 2;
    const int oh = h / stride, ow = w / stride;
    float* t = F(bf.t[li]);
    float* av = F(bf.a[li]);
    float* lv = F(bf.l[li]);
    // block 0: conv1 (stride) ; conv2 (+ fused 1x1/s2 downsample for li > 0)
    {
      ConvArgs a = conv_args(wb, p.blk[li][0][0], B, oh, ow, t, nullptr, 1);
      a.seg[0] = seg(xcur, B, h, w, cin, 3, stride, 1);
      io(a, xslot, -1, blk_slot(li, 0, 0));
      a.tile_cnt = TK(li, 0);
      a.tile_cnt_words = (int)bf.tick_words;
      SFA_RC(launch_conv(a, EPI_STD, m->math, st));
    }
    {
      ConvArgs a = conv_args(wb, p.blk[li][0][1], B, oh, ow, av, li == 0 ? xcur : nullptr, 1);
      a.seg[0] = seg(t, B, oh, ow, planes, 3, 1, 1);
      if (li > 0) {
        a.nseg = 2;
        a.kseg1 = 9 * planes;
        a.seg[1] = seg(xcur, B, h, w, cin, 1, stride, 0);
      }
      io(a, blk_slot(li, 0, 0), li > 0 ? xslot : -1, blk_slot(li, 0, 1));
      a.tile_cnt = TK(li, 1);
      a.tile_cnt_words = (int)bf.tick_words;
      SFA_RC(launch_conv(a, EPI_STD, m->math, st));
    }
    // block 1
    {
      ConvArgs a = conv_args(wb, p.blk[li][1][0], B, oh, ow, t, nullptr, 1);
      a.seg[0] = seg(av, B, oh, ow, planes, 3, 1, 1);
      io(a, blk_slot(li, 0, 1), -1, blk_slot(li, 1, 0));
      a.tile_cnt = TK(li, 2);
      a.tile_cnt_words = (int)bf.tick_words;
      SFA_RC(launch_conv(a, EPI_STD, m->math, st));
    }
    {
      ConvArgs a = conv_args(wb, p.blk[li][1][1], B, oh, ow, lv, av, 1);
      a.seg[0] = seg(t, B, oh, ow, planes, 3, 1, 1);
      io(a, blk_slot(li, 1, 0), -1, blk_slot(li, 1, 1));
      a.tile_cnt = TK(li, 3);
      a.tile_cnt_words = (int)bf.tick_words;
      SFA_RC(launch_conv(a, EPI_STD, m->math, st));
    }
    xcur = lv;
    xslot = blk_slot(li, 1, 1);
    h = oh;
    w = ow;
    cin = planes;
  }
  // FPN top-down (fpn_resnet.py:197-210): bilinear x2 (align_corners) + channel
  // concat, read by the 1x1 conv as two K-segments (no concat buffer).
  const int H4 = H / 4, W4 = W / 4, H8 = H / 8, W8 = W / 8, H16 = H / 16, W16 = W / 16;
  // fp16x3: each FPN 1x1 conv over cat(up(x), skip) runs as two convs on K-slices of its
  // packed weights, W_a up(x) + W_b skip + b = up(W_a x) + W_b skip + b (bilinear resize and a
  // 1x1 conv commute; the interpolation weights sum to 1): W_a x at the LOW resolution into a
  // half-res buffer (no bias), then W_b skip + b with that buffer added bilinearly upsampled in
  // the epilogue. A quarter of W_a's MACs, and up_level1 is never materialised.
  auto commute_at = [&](int f) { return h3 && ((m->fpn_commute >> f) & 1); };
  float* fpn_lo[3] = {F(bf.up1), F(bf.up1) + (size_t)B * (H / 32) * (W / 32) * 256,
                      F(bf.up1) + (size_t)B * (H / 32) * (W / 32) * 256 + (size_t)B * H16 * W16 * 128};
  auto fpn_pair = [&](int f, const float* x, int xh, int xw, int xc, int xslot_in, const float* skip, int sc,
                      int skip_slot, float* out, int out_slot, hipStream_t fs) -> int {
    const PConv& pc = p.fpn[f];
    {
      ConvArgs a = conv_args(wb, pc, B, xh, xw, fpn_lo[f], nullptr, 0);
      a.bias = nullptr;
      a.Kpad = xc;
      a.wstride = pc.Kpad;
      a.wk0 = 0;
      a.seg[0] = seg(x, B, xh, xw, xc, 1, 1, 0);
      a.fpn_gemm = (m->fpn_gemm >> f) & 1;
      io(a, xslot_in, -1, -1);
      SFA_RC(launch_conv(a, EPI_STD, m->math, fs));
    }
    ConvArgs a = conv_args(wb, pc, B, 2 * xh, 2 * xw, out, nullptr, 0);
    a.Kpad = sc;
    a.wstride = pc.Kpad;
    a.wk0 = xc;
    a.seg[0] = seg(skip, B, 2 * xh, 2 * xw, sc, 1, 1, 0);
    a.res_up = fpn_lo[f];
    a.res_sh = xh > 1 ? (float)(xh - 1) / (float)(2 * xh - 1) : 0.f;
    a.res_sw = xw > 1 ? (float)(xw - 1) / (float)(2 * xw - 1) : 0.f;
    a.fpn_gemm = (m->fpn_gemm >> (3 + f)) & 1;
    io(a, skip_slot, -1, out_slot);
    return launch_conv(a, EPI_STD, m->math, fs);
  };
  if (commute_at(0)) {
    SFA_RC(fpn_pair(0, F(bf.l[3]), H / 32, W / 32, 512, blk_slot(3, 1, 1), F(bf.l[2]), 256, blk_slot(2, 1, 1),
                    F(bf.c1), AM_FPN + 0, st));
  } else {
    SFA_RC(launch_upsample2x(F(bf.l[3]), F(bf.up1), B, H / 32, W / 32, 512, st));
    {
      ConvArgs a = conv_args(wb, p.fpn[0], B, H16, W16, F(bf.c1), nullptr, 0);
      a.nseg = 2;
      a.kseg1 = 512;
      a.seg[0] = seg(F(bf.up1), B, H16, W16, 512, 1, 1, 0);
      a.seg[1] = seg(F(bf.l[2]), B, H16, W16, 256, 1, 1, 0);
      io(a, blk_slot(3, 1, 1), blk_slot(2, 1, 1), AM_FPN + 0);  // up1 = upsample(layer4)
      SFA_RC(launch_conv(a, EPI_STD, m->math, st));
    }
  }
  SFA_RC(launch_upsample2x(F(bf.c1), F(bf.up2), B, H16, W16, 256, st));
  // Detection heads (fpn_resnet.py:219-233): per level all heads in one launch,
  // conv3x3 -> ReLU -> conv1x1 fused; channel-planar level outputs.
  int hoff[SFA_MAX_HEADS] = {0};
  int nch = 0;
  for (int j = 0; j < m->arch.num_heads; ++j) {
    hoff[j] = nch;
    nch += m->arch.head_channels[j];
  }
  const float* lin[3] = {F(bf.up2), F(bf.up3), F(bf.up4)};
  const int lh[3] = {H8, H4, H4}, lw[3] = {W8, W4, W4};
  float* lout[3] = {F(bf.L0), F(bf.L1), F(bf.L2)};
  auto head_args = [&](int f) -> ConvArgs {
    const PHeads& hp = p.heads[f];
    ConvArgs a;
    memset(&a, 0, sizeof a);
    a.nseg = 1;
    a.seg[0] = seg(lin[f], B, lh[f], lw[f], kFpnC[f], 3, 1, 1);
    a.Kpad = hp.K;
    a.w = wb + hp.w3;
    a.wx = reinterpret_cast<const uint16_t*>(wb + hp.wx);
    a.wh = reinterpret_cast<const uint16_t*>(wb + hp.wh);
    a.winv = wb + hp.winv;
    a.amax_in[0] = AM(AM_FPN + f);  // up2 / up3 / up4 come from conv_up_level1/2/3
    a.bias = wb + hp.b3;
    a.M = B * lh[f] * lw[f];
    a.N = hp.N;
    a.OH = lh[f];
    a.OW = lw[f];
    a.relu = 1;
    a.hw1 = wb + hp.w1;
    a.hb1 = wb + hp.b1;
    for (int j = 0; j < m->arch.num_heads; ++j) {
      a.hch[j] = m->arch.head_channels[j];
      a.hoff[j] = hoff[j];
    }
    a.hout = lout[f];
    return a;
  };
  auto probing = [&](hipStream_t hs) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    return (m->probe & SFA_PROBE_HEADS) && hipStreamIsCapturing(hs, &cap) == hipSuccess &&
           cap == hipStreamCaptureStatusNone;
  };
  auto launch_head = [&](int f, hipStream_t hs) -> int {
    const bool probe = probing(hs);
    if (probe) SFA_HIP_TRY(hipEventRecord(m->probe_ev[2 * f], hs));
    SFA_RC(launch_conv(head_args(f), EPI_HEAD, m->math, hs));
    if (probe) SFA_HIP_TRY(hipEventRecord(m->probe_ev[2 * f + 1], hs));
    return SFA_OK;
  };
  // (m->side is read under fork_mu below, as the overlap decision)
  // level 0 needs only up_level2: fork it onto the side stream (graph capture follows
  // the event edges), join before apply_kfpn
  // m->side is read under fork_mu: sfa_model_set_side_streams destroys it under the same lock,
  // so a concurrent call cannot pull a stream out from under this forward
  std::unique_lock<std::mutex> fork_lock(const_cast<sfa_model*>(m)->fork_mu);
  int sdev = -1;
  const bool overlap = m->side && !(m->probe & SFA_PROBE_SERIAL) &&
                       hipStreamGetDevice(st, &sdev) == hipSuccess && sdev == m->device;
  if (overlap) {
    SFA_HIP_TRY(hipEventRecord(m->fork, st));
    SFA_HIP_TRY(hipStreamWaitEvent(m->side, m->fork, 0));
  }
  // Everything between the fork and the join: any failure inside returns from this lambda
  // only, so the side stream is still joined below (a graph capture stays valid, no work is
  // left orphaned on the side stream).
  auto forked = [&]() -> int {
  SFA_RC(launch_head(0, overlap ? m->side : st));
  if (commute_at(1)) {
    SFA_RC(fpn_pair(1, F(bf.c1), H16, W16, 256, AM_FPN + 0, F(bf.l[1]), 128, blk_slot(1, 1, 1), F(bf.c2),
                    AM_FPN + 1, st));
  } else
  {
    ConvArgs a = conv_args(wb, p.fpn[1], B, H8, W8, F(bf.c2), nullptr, 0);
    a.nseg = 2;
    a.kseg1 = 256;
    a.seg[0] = seg(F(bf.up2), B, H8, W8, 256, 1, 1, 0);
    a.seg[1] = seg(F(bf.l[1]), B, H8, W8, 128, 1, 1, 0);
    io(a, AM_FPN + 0, blk_slot(1, 1, 1), AM_FPN + 1);
    SFA_RC(launch_conv(a, EPI_STD, m->math, st));
  }
  SFA_RC(launch_upsample2x(F(bf.c2), F(bf.up3), B, H8, W8, 128, st));
  // FPN level 3 (-> up_level4) on stream fs
  auto fpn3 = [&](hipStream_t fs) -> int {
    if (commute_at(2))
      return fpn_pair(2, F(bf.c2), H8, W8, 128, AM_FPN + 1, F(bf.l[0]), 64, blk_slot(0, 1, 1), F(bf.up4),
                      AM_FPN + 2, fs);
    ConvArgs a = conv_args(wb, p.fpn[2], B, H4, W4, F(bf.up4), nullptr, 0);
    a.nseg = 2;
    a.kseg1 = 128;
    a.seg[0] = seg(F(bf.up3), B, H4, W4, 128, 1, 1, 0);
    a.seg[1] = seg(F(bf.l[0]), B, H4, W4, 64, 1, 1, 0);
    io(a, AM_FPN + 1, blk_slot(0, 1, 1), AM_FPN + 2);
    return launch_conv(a, EPI_STD, m->math, fs);
  };
  SFA_RC(fpn3(st));
  // level 2 (needs up_level4, just written) on the side stream after level 0, level 1 here:
  // the two 1,444-tile launches run side by side, so neither one's last partial wave of tiles
  // leaves CUs idle
  if (overlap) {
    SFA_HIP_TRY(hipEventRecord(m->mid, st));
    SFA_HIP_TRY(hipStreamWaitEvent(m->side, m->mid, 0));
    SFA_RC(launch_head(2, m->side));
  }
  SFA_RC(launch_head(1, st));
  if (!overlap) SFA_RC(launch_head(2, st));
  return SFA_OK;
  };
  const int frc = forked();
  if (overlap) {  // the join, on success and on failure alike
    SFA_HIP_TRY(hipEventRecord(m->join, m->side));
    SFA_HIP_TRY(hipStreamWaitEvent(st, m->join, 0));
  }
  SFA_RC(frc);
  // apply_kfpn (fpn_resnet.py:248-254)
  KfpnOut ko;
  memset(&ko, 0, sizeof ko);
  for (int j = 0; j < m->arch.num_heads; ++j) {
    ko.ptr[j] = head_out[j];
    ko.ch[j] = m->arch.head_channels[j];
    ko.off[j] = hoff[j];
  }
  ko.num_heads = m->arch.num_heads;
  ko.total_ch = nch;
  SFA_RC(launch_kfpn(F(bf.L0), F(bf.L1), F(bf.L2), ko, B, H4, W4, st));
  return SFA_OK;
}

extern "C" int sfa_model_forward(const sfa_model* m, const float* x, int in_layout, int B, int H,
                                 int W, float* const* head_out, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  SFA_CHECK_ARG(m && x && head_out && workspace, "forward: null argument");
  SFA_CHECK_ARG(B >= 1 && H >= 32 && W >= 32 && H % 32 == 0 && W % 32 == 0,
                "forward: input (%d, 3, %d, %d) must have H, W multiples of 32", B, H, W);
  SFA_CHECK_ARG(in_layout == SFA_IN_NCHW3 || in_layout == SFA_IN_NHWC4 ||
                    in_layout == SFA_IN_NCHW3_FLIP_HW,
                "forward: bad layout");
  const int bmax = forward_max_batch(H, W);
  if (bmax < 1) {
    set_error("forward: one %d x %d frame exceeds the conv kernels' 32-bit buffer offsets", H, W);
    return SFA_E_UNSUPPORTED;
  }
  const int bc = std::min(B, bmax);
  const size_t need = plan_bufs(&m->arch, bc, H, W).total;
  if (workspace_bytes < need) {
    set_error("forward: workspace %zu < required %zu bytes", workspace_bytes, need);
    return SFA_E_WORKSPACE;
  }
  for (int j = 0; j < m->arch.num_heads; ++j) SFA_CHECK_ARG(head_out[j], "forward: null head out");
  // batches above the per-pass limit run as consecutive passes of bc frames on the caller's stream,
  // sharing the workspace (stream order serialises them)
  const size_t in_frame = (size_t)(in_layout == SFA_IN_NHWC4 ? 4 : 3) * H * W;
  const size_t out_px = (size_t)(H / 4) * (W / 4);
  float* outs[SFA_MAX_HEADS];
  for (int f0 = 0; f0 < B; f0 += bc) {
    const int nb = std::min(bc, B - f0);
    for (int j = 0; j < m->arch.num_heads; ++j)
      outs[j] = head_out[j] + (size_t)f0 * m->arch.head_channels[j] * out_px;
    SFA_RC(forward_pass(m, x + (size_t)f0 * in_frame, in_layout, nb, H, W, outs, workspace, stream));
  }
  return SFA_OK;
}
