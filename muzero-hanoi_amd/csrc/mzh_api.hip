// mzh_api.hip -- C ABI (include/mzh.h) over the gfx950 kernels.  No exceptions cross the ABI;
// every entry point returns a status and records a thread-local message.
#include <math.h>
#include <stdlib.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/mzh.h"
#include "mzh_env_kernels.h"
#include "mzh_internal.h"
#include "mzh_train.h"

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

static int hip_fail(hipError_t e, const char* what) {
  return fail(MZH_ERR_HIP, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
}

#define HIP_OK(expr)                                   \
  do {                                                 \
    hipError_t e_ = (expr);                            \
    if (e_ != hipSuccess) return hip_fail(e_, #expr);  \
  } while (0)

// RAII: run on the engine's device, restore the caller's current device afterwards
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

struct mzh_engine {
  int device = 0;
  int n_disks = 0, max_sims = 0, max_roots = 0, support = 33;
  int in_dim = 0, kin = 0, E = 0;
  void* wbuf = nullptr;
  bool loaded = false;
  MzhNet net{};
  MzhWNet wnet{};
  MzhOneNet onet{};
  unsigned char* tree = nullptr;
  float* htree = nullptr;
  uint16_t* pathx = nullptr;
  double* table = nullptr;
};

extern "C" int mzh_abi_version(void) { return MZH_ABI_VERSION; }
extern "C" const char* mzh_last_error(void) { return g_err.c_str(); }

extern "C" int mzh_device_count(int* count) {
  if (!count) return fail(MZH_ERR_ARG, "count is NULL");
  hipError_t e = hipGetDeviceCount(count);
  if (e != hipSuccess) {
    *count = 0;
    return hip_fail(e, "hipGetDeviceCount");
  }
  return MZH_OK;
}

extern "C" int mzh_host_device_pointer(void* host, void** dev) {
  if (!host || !dev) return fail(MZH_ERR_ARG, "host_device_pointer: NULL argument");
  *dev = nullptr;
  hipError_t e = hipHostGetDevicePointer(dev, host, 0);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "hipHostGetDevicePointer");
}

extern "C" int mzh_stream_synchronize(void* stream) {
  hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
  return e == hipSuccess ? MZH_OK : hip_fail(e, "hipStreamSynchronize");
}

static size_t canonical_size(int in_dim, int support) {
  const size_t H = MZH_LATENT, F = MZH_HIDDEN, A = MZH_ACTIONS;
  size_t s = 0;
  s += F * in_dim + F + H * F + H;
  s += F * (H + A) + F + H * F + H;
  s += F * H + F + (size_t)support * F + support;
  s += F * H + F + A * F + A;
  s += F * H + F + (size_t)support * F + support;
  return s;
}

extern "C" int mzh_weights_size(int n_disks, int support, size_t* n_floats) {
  if (n_disks < 1 || n_disks > 16 || (support != 33 && support != 1) || !n_floats)
    return fail(MZH_ERR_ARG, "bad n_disks=%d / support=%d", n_disks, support);
  *n_floats = canonical_size(3 * n_disks, support);
  return MZH_OK;
}

extern "C" int mzh_create(int device, int n_disks, int max_sims, int max_roots, int support, mzh_engine** out) {
  if (!out) return fail(MZH_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (n_disks < 1 || n_disks > 16) return fail(MZH_ERR_ARG, "n_disks must be in [1,16], got %d", n_disks);
  if (max_sims < 0 || max_sims > 32000) return fail(MZH_ERR_ARG, "max_sims must be in [0,32000], got %d", max_sims);
  if (max_roots < 1) return fail(MZH_ERR_ARG, "max_roots must be >= 1, got %d", max_roots);
  if (support != 33 && support != 1) return fail(MZH_ERR_ARG, "support must be 33 or 1, got %d", support);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MZH_ERR_HIP, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(MZH_ERR_ARG, "device %d out of range (%d devices)", device, ndev);
  DeviceGuard g(device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  mzh_engine* eng = new mzh_engine();
  eng->device = device;
  eng->n_disks = n_disks;
  eng->max_sims = max_sims;
  eng->max_roots = max_roots;
  eng->support = support;
  eng->in_dim = 3 * n_disks;
  eng->kin = ((eng->in_dim + 15) / 16) * 16;
  eng->E = max_sims + 1;
  const size_t nblk = (size_t)max_roots * eng->E;
  // MzhBlock (mzh_tree.h) / MzwBlock (mzh_wave.hip): one 128-B cache line per expanded node
  hipError_t e = hipMalloc(&eng->tree, nblk * 128);  // one 128-B block per expanded node
  if (e == hipSuccess) e = hipMalloc(&eng->htree, nblk * MZH_LATENT * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&eng->pathx, nblk * sizeof(uint16_t));
  if (e == hipSuccess) e = hipMalloc(&eng->table, sizeof(double) * (size_t)(max_sims + 2));
  if (e != hipSuccess) {
    mzh_destroy(eng);
    return hip_fail(e, "hipMalloc (engine workspace)");
  }
  // UCB table on the host with libm, exactly the reference's python expression (node.py:114-121)
  std::vector<double> t(max_sims + 2);
  for (int n = 0; n < max_sims + 2; ++n) t[n] = (log((double)(n + 19652 + 1) / 19652.0) + 1.25) * sqrt((double)n);
  e = hipMemcpy(eng->table, t.data(), sizeof(double) * t.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    mzh_destroy(eng);
    return hip_fail(e, "hipMemcpy (ucb table)");
  }
  *out = eng;
  return MZH_OK;
}

extern "C" int mzh_destroy(mzh_engine* eng) {
  if (!eng) return MZH_OK;
  DeviceGuard g(eng->device);
  if (eng->tree) (void)hipFree(eng->tree);
  if (eng->htree) (void)hipFree(eng->htree);
  if (eng->pathx) (void)hipFree(eng->pathx);
  if (eng->table) (void)hipFree(eng->table);
  if (eng->wbuf) (void)hipFree(eng->wbuf);
  delete eng;
  return MZH_OK;
}

// ---- weight packing: torch [N][K] -> MFMA fragment tiles (see MzhLayer in mzh_device.h) ----
struct PackedLayer {
  size_t woff = 0, boff = 0;  // float offsets into the device buffer
  int kb = 0, nt = 0;
};

static void pack_weights(std::vector<float>& buf, PackedLayer& L, const float* W, int N, int K, int ldw) {
  L.nt = (N + 15) / 16;
  L.kb = (K + 15) / 16;
  while (buf.size() % 4) buf.push_back(0.0f);
  L.woff = buf.size();
  buf.resize(buf.size() + (size_t)L.nt * L.kb * 64 * 4, 0.0f);
  float* dst = buf.data() + L.woff;
  for (int nt = 0; nt < L.nt; ++nt)
    for (int kb = 0; kb < L.kb; ++kb)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 4; ++j) {
          const int n = 16 * nt + (lane & 15);
          const int k = 16 * kb + 4 * j + (lane >> 4);
          dst[(((size_t)nt * L.kb + kb) * 64 + lane) * 4 + j] = (n < N && k < K) ? W[(size_t)n * ldw + k] : 0.0f;
        }
}
static void pack_bias(std::vector<float>& buf, PackedLayer& L, const float* b, int N) {
  while (buf.size() % 4) buf.push_back(0.0f);
  L.boff = buf.size();
  buf.resize(buf.size() + (size_t)L.nt * 16, 0.0f);
  for (int n = 0; n < N; ++n) buf[L.boff + n] = b[n];
}
static PackedLayer pack_layer(std::vector<float>& buf, const float* W, const float* b, int N, int K, int ldw) {
  PackedLayer L;
  pack_weights(buf, L, W, N, K, ldw);
  pack_bias(buf, L, b, N);
  return L;
}

// ---- wave-kernel packing (MzhWMlp, mzh_internal.h): weights as the MFMA A operand ----
static int wperm_u(int ht, int r) { return 16 * ht + 4 * (r & 3) + (r >> 2); }
enum WOut { WOUT_LATENT, WOUT_HEAD33, WOUT_NATURAL };
// output unit held by C row r (= 4g + i) of output tile ot, -1 for a padding row
static int wperm_out(WOut kind, int ot, int r, int n_out) {
  if (kind == WOUT_LATENT) return wperm_u(ot, r);
  if (kind == WOUT_HEAD33) {
    const int g = r >> 2, i = r & 3, sl = 4 * ot + i;
    const int k = 2 * g + (sl & 1) + 8 * (sl >> 1);  // partial q = 2g + (sl & 1), term sl >> 1
    return k < n_out ? k : -1;
  }
  const int k = 16 * ot + r;
  return k < n_out ? k : -1;
}
struct PackedW {
  size_t soff = 0, b1off = 0, b2off = 0, w32off = 0;
  float b32 = 0.0f;
  int kb1 = 0, no = 0;
};

// bin 32 of a 33-bin head (MzhNet::rwd32 / MzhWMlp::w32): [16 blocks b][4 chains g] float4
// {W2[32][16b + g], W2[32][16b + 4 + g], W2[32][16b + 8 + g], W2[32][16b + 12 + g]}
static size_t pack_bin32(std::vector<float>& buf, const float* W2) {
  while (buf.size() % 4) buf.push_back(0.0f);
  const size_t off = buf.size();
  buf.resize(buf.size() + 16 * 4 * 4, 0.0f);
  const float* row = W2 + (size_t)32 * MZH_HIDDEN;
  for (int b = 0; b < 16; ++b)
    for (int g = 0; g < 4; ++g)
      for (int t = 0; t < 4; ++t) buf[off + (size_t)(b * 4 + g) * 4 + t] = row[16 * b + 4 * t + g];
  return off;
}
static PackedW pack_wmlp(std::vector<float>& buf, const float* W1, const float* b1, int K1, int ldw1, const float* W2,
                         const float* b2, int n_out, WOut kind) {
  PackedW P;
  P.kb1 = (K1 + 15) / 16;
  // a 33-bin head keeps bins 0..31 in two tiles; bin 32 goes to the vector chains (pack_bin32)
  P.no = kind == WOUT_HEAD33 ? 2 : (n_out + 15) / 16;
  const int FR = P.kb1 + P.no;
  while (buf.size() % 4) buf.push_back(0.0f);
  P.soff = buf.size();
  buf.resize(buf.size() + (size_t)17 * FR * 64 * 4, 0.0f);  // ht block 16 = zero pad
  float* s = buf.data() + P.soff;
  for (int ht = 0; ht < 16; ++ht)
    for (int lane = 0; lane < 64; ++lane)
      for (int t = 0; t < 4; ++t) {
        const int r = lane & 15, gk = lane >> 4;
        for (int kb = 0; kb < P.kb1; ++kb) {
          const int k = 16 * kb + 4 * t + gk;
          s[(((size_t)ht * FR + kb) * 64 + lane) * 4 + t] = k < K1 ? W1[(size_t)wperm_u(ht, r) * ldw1 + k] : 0.0f;
        }
        for (int ot = 0; ot < P.no; ++ot) {
          const int row = wperm_out(kind, ot, r, n_out);
          const int k = 16 * ht + 4 * t + gk;
          s[(((size_t)ht * FR + P.kb1 + ot) * 64 + lane) * 4 + t] = row >= 0 ? W2[(size_t)row * MZH_HIDDEN + k] : 0.0f;
        }
      }
  P.b1off = buf.size();
  buf.resize(buf.size() + MZH_HIDDEN, 0.0f);
  for (int ht = 0; ht < 16; ++ht)
    for (int r = 0; r < 16; ++r) buf[P.b1off + 16 * ht + r] = b1[wperm_u(ht, r)];
  P.b2off = buf.size();
  buf.resize(buf.size() + (size_t)16 * P.no, 0.0f);
  for (int ot = 0; ot < P.no; ++ot)
    for (int r = 0; r < 16; ++r) {
      const int row = wperm_out(kind, ot, r, n_out);
      buf[P.b2off + 16 * ot + r] = row >= 0 ? b2[row] : 0.0f;
    }
  while (buf.size() % 4) buf.push_back(0.0f);
  if (kind == WOUT_HEAD33) {
    P.w32off = pack_bin32(buf, W2);
    P.b32 = b2[32];
  }
  return P;
}

// ---- latency-path packing (MzhOneNet, mzh_internal.h): float offsets of its arrays in the blob ----
struct PackedOne {
  size_t l1 = 0, b1 = 0, rep0 = 0, rep0b = 0, rep2 = 0, rep2b = 0, l2 = 0;
};
static PackedOne pack_one(std::vector<float>& buf, int in, int sup, const float* rep0w, const float* rep0b,
                          const float* rep2w, const float* rep2b, const float* dyn0w, const float* dyn0b,
                          const float* dyn2w, const float* dyn2b, const float* rwd0w, const float* rwd0b,
                          const float* rwd2w, const float* rwd2b, const float* pol0w, const float* pol0b,
                          const float* pol2w, const float* pol2b, const float* val0w, const float* val0b,
                          const float* val2w, const float* val2b) {
  const int H = MZH_LATENT, F = MZH_HIDDEN, A = MZH_ACTIONS;
  auto align4 = [&]() { while (buf.size() % 4) buf.push_back(0.0f); };
  PackedOne o;
  // l1 [66 k4][256 units] float4
  align4();
  o.l1 = buf.size();
  buf.resize(buf.size() + (size_t)66 * F * 4, 0.0f);
  for (int k4 = 0; k4 < 66; ++k4)
    for (int u = 0; u < F; ++u)
      for (int i = 0; i < 4; ++i) {
        float v = 0.0f;
        if (k4 < 16) v = dyn0w[(size_t)u * (H + A) + 4 * k4 + i];
        else if (k4 < 32) v = rwd0w[(size_t)u * H + 4 * (k4 - 16) + i];
        else if (k4 < 48) v = pol0w[(size_t)u * H + 4 * (k4 - 32) + i];
        else if (k4 < 64) v = val0w[(size_t)u * H + 4 * (k4 - 48) + i];
        else if (4 * (k4 - 64) + i < A) v = dyn0w[(size_t)u * (H + A) + H + 4 * (k4 - 64) + i];
        buf[o.l1 + ((size_t)k4 * F + u) * 4 + i] = v;
      }
  o.b1 = buf.size();
  buf.resize(buf.size() + (size_t)F * 4);
  for (int u = 0; u < F; ++u) {
    buf[o.b1 + 4 * u] = dyn0b[u];
    buf[o.b1 + 4 * u + 1] = rwd0b[u];
    buf[o.b1 + 4 * u + 2] = pol0b[u];
    buf[o.b1 + 4 * u + 3] = val0b[u];
  }
  // representation_net.0 k-major [in][256], its bias; representation_net.2 [64 k4][64] float4, its bias
  o.rep0 = buf.size();
  buf.resize(buf.size() + (size_t)in * F);
  for (int k = 0; k < in; ++k)
    for (int u = 0; u < F; ++u) buf[o.rep0 + (size_t)k * F + u] = rep0w[(size_t)u * in + k];
  o.rep0b = buf.size();
  buf.insert(buf.end(), rep0b, rep0b + F);
  align4();
  o.rep2 = buf.size();
  buf.resize(buf.size() + (size_t)64 * 64 * 4);
  for (int k4 = 0; k4 < 64; ++k4)
    for (int j = 0; j < 64; ++j)
      for (int i = 0; i < 4; ++i) buf[o.rep2 + ((size_t)k4 * 64 + j) * 4 + i] = rep2w[(size_t)j * F + 4 * k4 + i];
  o.rep2b = buf.size();
  buf.insert(buf.end(), rep2b, rep2b + H);
  // the LDS image
  align4();
  o.l2 = buf.size();
  buf.resize(buf.size() + (size_t)MZH_ONE_L2F4 * 4, 0.0f);
  float* L = buf.data() + o.l2;
  const int nb = sup < 32 ? sup : 32;  // bins of each head in the A2 rows
  for (int k4 = 0; k4 < 64; ++k4)
    for (int j = 0; j < 64; ++j)
      for (int i = 0; i < 4; ++i) {
        const int k = 4 * k4 + i;
        L[((size_t)MZH_ONE_D2 + k4 * 64 + j) * 4 + i] = dyn2w[(size_t)j * F + k];
        const int row = j & 31;
        const float* W2 = j < 32 ? rwd2w : val2w;
        L[((size_t)MZH_ONE_A2 + k4 * 64 + j) * 4 + i] = row < nb ? W2[(size_t)row * F + k] : 0.0f;
        if (j < 8) L[((size_t)MZH_ONE_P2 + k4 * 8 + j) * 4 + i] = j < A ? pol2w[(size_t)j * F + k] : 0.0f;
      }
  if (sup == 33)
    for (int i = 0; i < 64; ++i)
      for (int ln = 0; ln < 8; ++ln) {
        const float* W2 = ln < 4 ? rwd2w : val2w;
        L[(size_t)MZH_ONE_C32 * 4 + ln * 64 + i] = W2[(size_t)32 * F + (ln & 3) + 4 * i];
      }
  float* B2 = L + (size_t)MZH_ONE_B2 * 4;
  for (int j = 0; j < 64; ++j) {
    B2[j] = dyn2b[j];
    B2[64 + j] = (j & 31) < nb ? (j < 32 ? rwd2b : val2b)[j & 31] : 0.0f;
  }
  for (int j = 0; j < A; ++j) B2[128 + j] = pol2b[j];
  if (sup == 33) {
    B2[136] = rwd2b[32];
    B2[137] = val2b[32];
  }
  return o;
}

extern "C" int mzh_load_weights(mzh_engine* eng, const float* flat, size_t n_floats) {
  if (!eng || !flat) return fail(MZH_ERR_ARG, "engine or weights NULL");
  const size_t want = canonical_size(eng->in_dim, eng->support);
  if (n_floats != want) return fail(MZH_ERR_ARG, "weights: expected %zu floats, got %zu", want, n_floats);
  const int H = MZH_LATENT, F = MZH_HIDDEN, A = MZH_ACTIONS, in = eng->in_dim, sup = eng->support;
  const float* p = flat;
  auto take = [&](size_t n) { const float* q = p; p += n; return q; };
  const float *rep0w = take((size_t)F * in), *rep0b = take(F), *rep2w = take((size_t)H * F), *rep2b = take(H);
  const float *dyn0w = take((size_t)F * (H + A)), *dyn0b = take(F), *dyn2w = take((size_t)H * F), *dyn2b = take(H);
  const float *rwd0w = take((size_t)F * H), *rwd0b = take(F), *rwd2w = take((size_t)sup * F), *rwd2b = take(sup);
  const float *pol0w = take((size_t)F * H), *pol0b = take(F), *pol2w = take((size_t)A * F), *pol2b = take(A);
  const float *val0w = take((size_t)F * H), *val0b = take(F), *val2w = take((size_t)sup * F), *val2b = take(sup);

  std::vector<float> buf;
  buf.reserve(200000);
  PackedLayer L[10];
  L[0] = pack_layer(buf, rep0w, rep0b, F, in, in);
  L[1] = pack_layer(buf, rep2w, rep2b, H, F, F);
  L[2] = pack_layer(buf, dyn0w, dyn0b, F, H, H + A);  // h part only (k < 64)
  L[3] = pack_layer(buf, dyn2w, dyn2b, H, F, F);
  L[4] = pack_layer(buf, rwd0w, rwd0b, F, H, H);
  // 33-bin heads: bins 0..31 as MFMA tiles, bin 32 by vector chains (MzhNet::rwd32 / val32)
  const int nhead = sup == 33 ? 32 : sup;
  L[5] = pack_layer(buf, rwd2w, rwd2b, nhead, F, F);
  // pol0 and val0 weights back to back: the search kernel's prediction chunks take consecutive
  // tiles of this 32-tile strip and load them as one contiguous run (mzh_mma_store ring refill)
  pack_weights(buf, L[6], pol0w, F, H, H);
  pack_weights(buf, L[8], val0w, F, H, H);
  pack_bias(buf, L[6], pol0b, F);
  pack_bias(buf, L[8], val0b, F);
  L[7] = pack_layer(buf, pol2w, pol2b, A, F, F);
  L[9] = pack_layer(buf, val2w, val2b, nhead, F, F);
  while (buf.size() % 4) buf.push_back(0.0f);
  const size_t ohoff = buf.size();
  buf.resize(buf.size() + (size_t)A * F);
  for (int a = 0; a < A; ++a)
    for (int n = 0; n < F; ++n) buf[ohoff + (size_t)a * F + n] = dyn0w[(size_t)n * (H + A) + H + a];
  // wave-kernel layout
  const WOut vkind = sup == 33 ? WOUT_HEAD33 : WOUT_NATURAL;
  PackedW WL[5];
  WL[0] = pack_wmlp(buf, rep0w, rep0b, in, in, rep2w, rep2b, H, WOUT_LATENT);
  WL[1] = pack_wmlp(buf, dyn0w, dyn0b, H, H + A, dyn2w, dyn2b, H, WOUT_LATENT);
  WL[2] = pack_wmlp(buf, rwd0w, rwd0b, H, H, rwd2w, rwd2b, sup, vkind);
  WL[3] = pack_wmlp(buf, pol0w, pol0b, H, H, pol2w, pol2b, A, WOUT_NATURAL);
  WL[4] = pack_wmlp(buf, val0w, val0b, H, H, val2w, val2b, sup, vkind);
  const size_t wohoff = buf.size();
  buf.resize(buf.size() + (size_t)A * F, 0.0f);
  for (int a = 0; a < A; ++a)
    for (int j = 0; j < F; ++j) buf[wohoff + (size_t)a * F + j] = dyn0w[(size_t)wperm_u(j >> 4, j & 15) * (H + A) + H + a];
  // latency-path layout
  const PackedOne PO = pack_one(buf, in, sup, rep0w, rep0b, rep2w, rep2b, dyn0w, dyn0b, dyn2w, dyn2b, rwd0w, rwd0b,
                                rwd2w, rwd2b, pol0w, pol0b, pol2w, pol2b, val0w, val0b, val2w, val2b);

  DeviceGuard g(eng->device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  if (eng->wbuf) {
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipFree(eng->wbuf));
    eng->wbuf = nullptr;
    eng->loaded = false;
  }
  HIP_OK(hipMalloc(&eng->wbuf, buf.size() * sizeof(float)));
  HIP_OK(hipMemcpy(eng->wbuf, buf.data(), buf.size() * sizeof(float), hipMemcpyHostToDevice));
  const float* base = static_cast<const float*>(eng->wbuf);
  auto mk = [&](const PackedLayer& pl) {
    MzhLayer m;
    m.w = reinterpret_cast<const float4*>(base + pl.woff);
    m.b = base + pl.boff;
    m.kb = pl.kb;
    m.nt = pl.nt;
    m.woff = (int)(pl.woff * sizeof(float));
    m.boff = (int)(pl.boff * sizeof(float));
    return m;
  };
  MzhNet& n = eng->net;
  n.wbase = base;
  n.rep0 = mk(L[0]); n.rep2 = mk(L[1]); n.dyn0 = mk(L[2]); n.dyn2 = mk(L[3]); n.rwd0 = mk(L[4]);
  n.rwd2 = mk(L[5]); n.pol0 = mk(L[6]); n.pol2 = mk(L[7]); n.val0 = mk(L[8]); n.val2 = mk(L[9]);
  if (n.val0.w != n.pol0.w + (size_t)n.pol0.nt * n.pol0.kb * 64)
    return fail(MZH_ERR_STATE, "pol0/val0 weights not contiguous");
  n.dyn0_onehot = base + ohoff;
  n.rwd32 = n.val32 = nullptr;
  n.rwd32b = n.val32b = 0.0f;
  if (sup == 33) {  // the wave layout's bin-32 arrays serve both kernels
    n.rwd32 = reinterpret_cast<const float4*>(base + WL[2].w32off);
    n.val32 = reinterpret_cast<const float4*>(base + WL[4].w32off);
    n.rwd32b = WL[2].b32;
    n.val32b = WL[4].b32;
  }
  n.support = sup;
  n.in_dim = in;
  auto mkw = [&](const PackedW& pw) {
    MzhWMlp m;
    m.s = reinterpret_cast<const float4*>(base + pw.soff);
    m.b1 = base + pw.b1off;
    m.b2 = base + pw.b2off;
    m.kb1 = pw.kb1;
    m.no = pw.no;
    m.w32 = pw.w32off ? reinterpret_cast<const float4*>(base + pw.w32off) : nullptr;
    m.b32 = pw.b32;
    m.soff = (int)(pw.soff * sizeof(float));
    m.b1off = (int)(pw.b1off * sizeof(float));
    m.b2off = (int)(pw.b2off * sizeof(float));
    m.w32off = (int)(pw.w32off * sizeof(float));
    return m;
  };
  MzhWNet& w = eng->wnet;
  w.wbase = base;
  w.rep = mkw(WL[0]); w.dyn = mkw(WL[1]); w.rwd = mkw(WL[2]); w.pol = mkw(WL[3]); w.val = mkw(WL[4]);
  w.oh = base + wohoff;
  w.support = sup;
  w.in_dim = in;
  MzhOneNet& o = eng->onet;
  o.l1 = reinterpret_cast<const float4*>(base + PO.l1);
  o.b1 = reinterpret_cast<const float4*>(base + PO.b1);
  o.rep0 = base + PO.rep0;
  o.rep0b = base + PO.rep0b;
  o.rep2 = reinterpret_cast<const float4*>(base + PO.rep2);
  o.rep2b = base + PO.rep2b;
  o.l2 = reinterpret_cast<const float4*>(base + PO.l2);
  eng->loaded = true;
  return MZH_OK;
}

// ---- environment ----
extern "C" int mzh_env_step(int n_disks, int goal_peg, int max_steps, int B, uint8_t* state, const int32_t* action,
                            uint8_t* moved, float* obs, int8_t* reward, uint8_t* done, uint8_t* illegal,
                            int32_t* step_ctr, uint8_t* active, int32_t* err_count, mzh_stream stream) {
  if (n_disks < 1 || n_disks > 32 || goal_peg < 0 || goal_peg > 2 || B < 0)
    return fail(MZH_ERR_ARG, "env_step: bad n_disks=%d goal_peg=%d B=%d", n_disks, goal_peg, B);
  if (B == 0) return MZH_OK;
  if (!state || !action || !reward || !done || !illegal || !step_ctr || !active)
    return fail(MZH_ERR_ARG, "env_step: required buffer is NULL");
  hipError_t e = mzh_launch_env_step(n_disks, goal_peg, max_steps, B, state, action, moved, obs, reward, done, illegal,
                                     step_ctr, active, err_count, (hipStream_t)stream);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "env_step launch");
}

extern "C" int mzh_legal_mask(int n_disks, int B, const uint8_t* state, uint8_t* mask, mzh_stream stream) {
  if (n_disks < 1 || n_disks > 32 || B < 0 || (B > 0 && (!state || !mask))) return fail(MZH_ERR_ARG, "legal_mask: bad args");
  if (B == 0) return MZH_OK;
  hipError_t e = mzh_launch_legal_mask(n_disks, B, state, mask, (hipStream_t)stream);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "legal_mask launch");
}

extern "C" int mzh_encode_obs(int n_disks, int B, const uint8_t* state, float* obs, mzh_stream stream) {
  if (n_disks < 1 || n_disks > 32 || B < 0 || (B > 0 && (!state || !obs))) return fail(MZH_ERR_ARG, "encode_obs: bad args");
  if (B == 0) return MZH_OK;
  hipError_t e = mzh_launch_encode_obs(n_disks, B, state, obs, (hipStream_t)stream);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "encode_obs launch");
}

extern "C" int mzh_hanoi_solver(int n_disks, int goal_peg, int B, const uint8_t* state, int32_t* moves, mzh_stream stream) {
  if (n_disks < 1 || n_disks > 30 || goal_peg < 0 || goal_peg > 2 || B < 0 || (B > 0 && (!state || !moves)))
    return fail(MZH_ERR_ARG, "hanoi_solver: bad args");
  if (B == 0) return MZH_OK;
  hipError_t e = mzh_launch_hanoi_solver(n_disks, goal_peg, B, state, moves, (hipStream_t)stream);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "hanoi_solver launch");
}

// ---- inference ----
// roots (rows) per workgroup of the standalone inference kernels: 16 while that fits one workgroup
// per CU (B <= 4096), else 32
static int pick_rows(int B) { return B > 256 * 16 ? 32 : 16; }

// cooperative search tile: 16 roots while that is one round of workgroups (B <= 4,096), else 32
// roots (a second round of 16-root workgroups costs more than 32-root tiles).  MZH_FLAG_COOP_TILE16 /
// MZH_FLAG_COOP_TILE32 force one (tests reach both tiles' code paths at any batch size).
static int pick_tile(int B, uint32_t flags) {
  if (flags & MZH_FLAG_COOP_TILE16) return 16;
  if (flags & MZH_FLAG_COOP_TILE32) return 32;
  return B > 256 * 16 ? 32 : 16;
}

extern "C" int mzh_initial_inference(mzh_engine* eng, int B, const float* obs, float* h, float* reward, float* pi,
                                     float* value, float* policy_logits, float* value_logits, mzh_stream stream) {
  if (!eng) return fail(MZH_ERR_ARG, "engine NULL");
  if (!eng->loaded) return fail(MZH_ERR_STATE, "weights not loaded");
  if (B < 0 || (B > 0 && (!obs || !h))) return fail(MZH_ERR_ARG, "initial_inference: bad args");
  if (B == 0) return MZH_OK;
  DeviceGuard g(eng->device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  MzhInferParams p{};
  p.B = B; p.in_dim = eng->in_dim; p.kin = eng->kin; p.x = obs; p.h = h; p.reward = reward; p.pi = pi;
  p.value = value; p.policy_logits = policy_logits; p.value_logits = value_logits;
  hipError_t e = mzh_launch_infer(pick_rows(B), false, eng->net, p, (hipStream_t)stream);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "initial_inference launch");
}

extern "C" int mzh_recurrent_inference(mzh_engine* eng, int B, const float* h_in, const int32_t* action, float* h,
                                       float* reward, float* pi, float* value, float* policy_logits,
                                       float* value_logits, float* reward_logits, mzh_stream stream) {
  if (!eng) return fail(MZH_ERR_ARG, "engine NULL");
  if (!eng->loaded) return fail(MZH_ERR_STATE, "weights not loaded");
  if (B < 0 || (B > 0 && (!h_in || !action || !h))) return fail(MZH_ERR_ARG, "recurrent_inference: bad args");
  if (B == 0) return MZH_OK;
  DeviceGuard g(eng->device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  MzhInferParams p{};
  p.B = B; p.in_dim = eng->in_dim; p.kin = eng->kin; p.x = h_in; p.action = action; p.h = h; p.reward = reward;
  p.pi = pi; p.value = value; p.policy_logits = policy_logits; p.value_logits = value_logits;
  p.reward_logits = reward_logits;
  hipError_t e = mzh_launch_infer(pick_rows(B), true, eng->net, p, (hipStream_t)stream);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "recurrent_inference launch");
}

// ---- search ----
static const size_t kMaxLds = 163840;

// kernel choice: the wave-independent kernel (mzh_wave.hip) with 32 roots per wave once the batch
// gives two such waves per SIMD, with 16 roots per wave for mid-size batches (>= 1024 such waves),
// else the cooperative kernel (mzh_search.hip) whose 4 waves split every MLP layer of one 16- or
// 32-root tile.  MZH_FLAG_KERNEL_* (or MZH_KERNEL=coop|wave|wave16) force one.
static const int kWaveMinRoots = 53248, kWave16MinRoots = 8193;  // measured crossovers
struct KernelChoice {
  bool wave;
  int nt;  // wave kernel: 16-root column tiles per wave
};
static KernelChoice choose_kernel(int B, uint32_t flags) {
  if (flags & MZH_FLAG_KERNEL_WAVE16) return {true, 1};
  if (flags & MZH_FLAG_KERNEL_WAVE) return {true, 2};
  if (flags & MZH_FLAG_KERNEL_COOP) return {false, 0};
  static const int forced = [] {
    const char* v = getenv("MZH_KERNEL");
    if (!v) return 0;
    return strcmp(v, "wave") == 0 ? 2 : strcmp(v, "wave16") == 0 ? 1 : strcmp(v, "coop") == 0 ? -1 : 0;
  }();
  if (forced) return forced > 0 ? KernelChoice{true, forced} : KernelChoice{false, 0};
  if (B >= kWaveMinRoots) return {true, 2};
  if (B >= kWave16MinRoots) return {true, 1};
  return {false, 0};
}

// the latency path (mzh_one.hip): MLP searches of up to kOneMaxRoots roots take one root per workgroup
// (persistent over the roots beyond the 256 workgroups of one round) while its LDS fits; a forced kernel
// flag (or MZH_KERNEL) decides otherwise.  MZH_FLAG_KERNEL_ONE forces it (an error where it cannot run).
static const int kOneMaxRoots = 512, kOneGrid = 256;  // crossover: profiles/r06_one_probe.json
static bool one_forced_env() {
  static const bool f = [] {
    const char* v = getenv("MZH_KERNEL");
    return v && strcmp(v, "one") == 0;
  }();
  return f;
}

// every template argument of the launch (MzhSearchPlan); returns a status (capacity errors)
static int make_plan(int B, int S, uint32_t flags, bool replay, int support, bool has_minmax, MzhSearchPlan* pl) {
  const uint32_t forced = flags & (MZH_FLAG_KERNEL_COOP | MZH_FLAG_KERNEL_WAVE | MZH_FLAG_KERNEL_WAVE16 | MZH_FLAG_COOP_OCC2 |
                                   MZH_FLAG_COOP_TILE16 | MZH_FLAG_COOP_TILE32);
  const bool one_fits = mzh_one_smem_bytes(S, false) <= kMaxLds;
  if (flags & MZH_FLAG_KERNEL_ONE) {
    if (replay) return fail(MZH_ERR_ARG, "MZH_FLAG_KERNEL_ONE: the latency kernel has no replay (tree-only) form");
    if (forced) return fail(MZH_ERR_ARG, "MZH_FLAG_KERNEL_ONE combined with another kernel flag");
    if (!one_fits)
      return fail(MZH_ERR_CAPACITY, "MZH_FLAG_KERNEL_ONE: n_sims=%d needs %zu B of LDS", S, mzh_one_smem_bytes(S, false));
  }
  const bool env_kernel = getenv("MZH_KERNEL") != nullptr;
  if (!replay && one_fits &&
      ((flags & MZH_FLAG_KERNEL_ONE) || one_forced_env() || (!forced && !env_kernel && B <= kOneMaxRoots))) {
    MzhSearchPlan q{};
    q.one = 1;
    q.ohl = mzh_one_smem_bytes(S, true) <= kMaxLds;  // the latents in LDS where they fit
    q.sup33 = support == 33;
    q.mmin = has_minmax ? 1 : 0;
    q.grid = B < kOneGrid ? B : kOneGrid;
    *pl = q;
    return MZH_OK;
  }
  const KernelChoice kc = choose_kernel(B, flags);
  MzhSearchPlan q{};
  q.wave = kc.wave ? 1 : 0;
  q.nt = kc.nt;
  q.replay = replay ? 1 : 0;
  q.mmin = has_minmax ? 1 : 0;
  if (kc.wave) {
    if (mzh_wave_smem_bytes(S, kc.nt) > kMaxLds)
      return fail(MZH_ERR_CAPACITY, "n_sims=%d exceeds the wave kernel's LDS table budget", S);
    q.sup33 = support == 33;
    q.mmin = 0;  // the wave kernel decides the exact normaliser per selection
  } else {
    q.R = pick_tile(B, flags);
    // the two-workgroups-per-CU 16-root kernel: forced by MZH_FLAG_COOP_OCC2 (MLP searches; its LDS must
    // leave room for the second workgroup -- a search it cannot serve is an error, never a silent fallback;
    // replay searches have no occ2 instantiation and take the cooperative replay kernel, as mzh.h says)
    if ((flags & MZH_FLAG_COOP_OCC2) && !replay && 2 * mzh_search_smem_bytes(16, S, false, true) > kMaxLds)
      return fail(MZH_ERR_CAPACITY, "MZH_FLAG_COOP_OCC2: n_sims=%d needs %zu B of LDS per workgroup, more than "
                  "half a CU's", S, mzh_search_smem_bytes(16, S, false, true));
    if ((flags & MZH_FLAG_COOP_OCC2) && !replay) {
      q.R = 16;
      q.occ2 = 1;
      q.ohl = 0;
      q.sup33 = support == 33;
      *pl = q;
      return MZH_OK;
    }
    if (mzh_search_smem_bytes(q.R, S, false) > kMaxLds) q.R = 16;
    if (mzh_search_smem_bytes(q.R, S, false) > kMaxLds)
      return fail(MZH_ERR_CAPACITY, "n_sims=%d exceeds the LDS path budget", S);
    // the one-hot columns go to LDS when they fit (never in the replay kernel, which runs no MLP)
    q.ohl = !replay && mzh_search_smem_bytes(q.R, S, true) <= kMaxLds;
    q.sup33 = replay || support == 33;
  }
  *pl = q;
  return MZH_OK;
}

static void plan_info(const MzhSearchPlan& q, int B, int S, mzh_search_plan* out) {
  memset(out, 0, sizeof(*out));
  const char* tf[2] = {"false", "true"};
  out->wave = q.wave;
  if (q.one) {
    out->roots_per_wave = 1;
    out->threads_per_workgroup = 512;
    out->roots_per_workgroup = 1;
    out->smem_bytes = (int64_t)mzh_one_smem_bytes(S, q.ohl);
    snprintf(out->kernel, sizeof(out->kernel), "mzh_search_one_kernel<%s, %s, %s>", tf[q.sup33], tf[q.mmin], tf[q.ohl]);
    out->workgroups = q.grid;
    return;
  }
  if (q.wave) {
    out->roots_per_wave = 16 * q.nt;
    out->threads_per_workgroup = 256;
    out->roots_per_workgroup = 4 * 16 * q.nt;
    out->smem_bytes = (int64_t)mzh_wave_smem_bytes(S, q.nt);
    snprintf(out->kernel, sizeof(out->kernel), "mzh_wave_kernel<%d, %s, %s>", q.nt, tf[q.replay], tf[q.sup33]);
  } else if (q.occ2) {
    out->roots_per_wave = 4;
    out->threads_per_workgroup = MZH_THREADS;
    out->roots_per_workgroup = 16;
    out->smem_bytes = (int64_t)mzh_search_smem_bytes(16, S, false, true);
    snprintf(out->kernel, sizeof(out->kernel), "mzh_search_occ2_kernel<%s, %s>", tf[q.sup33], tf[q.mmin]);
  } else {
    out->roots_per_wave = q.R / 4;
    out->threads_per_workgroup = MZH_THREADS;
    out->roots_per_workgroup = q.R;
    out->smem_bytes = (int64_t)mzh_search_smem_bytes(q.R, S, q.ohl);
    snprintf(out->kernel, sizeof(out->kernel), "mzh_search_kernel<%d, %s, %s, %s, %s>", q.R, tf[q.replay], tf[q.ohl],
             tf[q.sup33], tf[q.mmin]);
  }
  out->workgroups = (B + out->roots_per_workgroup - 1) / out->roots_per_workgroup;
}

extern "C" int mzh_search_plan_query(int support, int B, int n_sims, uint32_t flags, int replay, int has_minmax_in,
                                     mzh_search_plan* out) {
  if (!out) return fail(MZH_ERR_ARG, "out is NULL");
  if (B < 1 || n_sims < 0 || n_sims > 32000 || (support != 33 && support != 1))
    return fail(MZH_ERR_ARG, "search_plan: bad B=%d n_sims=%d support=%d", B, n_sims, support);
  MzhSearchPlan q;
  const int st = make_plan(B, n_sims, flags, replay != 0, support, has_minmax_in != 0, &q);
  if (st) return st;
  plan_info(q, B, n_sims, out);
  return MZH_OK;
}

static int search_common(mzh_engine* eng, const mzh_search_args* a, mzh_stream stream, bool replay) {
  if (!eng || !a) return fail(MZH_ERR_ARG, "engine or args NULL");
  if (a->B < 0 || a->n_sims < 0) return fail(MZH_ERR_ARG, "B=%d n_sims=%d", a->B, a->n_sims);
  if (a->B > eng->max_roots) return fail(MZH_ERR_CAPACITY, "B=%d > max_roots=%d", a->B, eng->max_roots);
  if (a->n_sims > eng->max_sims) return fail(MZH_ERR_CAPACITY, "n_sims=%d > max_sims=%d", a->n_sims, eng->max_sims);
  if (!(a->temperature >= 0.0 && a->temperature <= 1.0))
    return fail(MZH_ERR_TEMPERATURE, "Expect `temperature` to be in the range [0.0, 1.0], got %g", a->temperature);
  if (a->B == 0) {  // nothing launches: the plan says so (a caller naming the kernel sees "none")
    if (a->plan_out) {
      memset(a->plan_out, 0, sizeof(*a->plan_out));
      snprintf(a->plan_out->kernel, sizeof(a->plan_out->kernel), "none");
    }
    return MZH_OK;
  }
  if (!a->visits) return fail(MZH_ERR_ARG, "visits output is required");
  if (replay) {
    if (!a->rp_root_pi || (a->n_sims > 0 && !a->rp_sim))
      return fail(MZH_ERR_ARG, "replay search needs rp_root_pi and rp_sim");
  } else {
    if (!eng->loaded) return fail(MZH_ERR_STATE, "weights not loaded");
    if (!a->obs) return fail(MZH_ERR_ARG, "obs is required");
  }
  if (!a->deterministic && !a->action_u && a->action)
    return fail(MZH_ERR_ARG, "stochastic action selection needs action_u");
  MzhSearchPlan pl;
  const int st = make_plan(a->B, a->n_sims, a->flags, replay, eng->support, a->minmax_in != nullptr, &pl);
  if (st) return st;
  if (a->plan_out) plan_info(pl, a->B, a->n_sims, a->plan_out);
  DeviceGuard g(eng->device);
  if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
  MzhSearchParams p{};
  p.B = a->B; p.S = a->n_sims; p.E = eng->E; p.in_dim = eng->in_dim; p.kin = eng->kin;
  p.deterministic = a->deterministic; p.np1 = (a->flags & MZH_FLAG_NP1_UCB) ? 1 : 0;
  p.discount = a->discount; p.eps = a->eps; p.temperature = a->temperature;
  p.obs = a->obs; p.noise = a->noise; p.tie_idx = a->tie_idx; p.action_u = a->action_u; p.minmax_in = a->minmax_in;
  p.rp_root_pi = a->rp_root_pi; p.rp_sim = a->rp_sim;
  p.tree = eng->tree; p.htree = eng->htree; p.pathx = eng->pathx; p.table = eng->table;
  p.visits = a->visits; p.root_q = a->root_q; p.minmax_out = a->minmax_out; p.extra_ties = a->extra_ties;
  p.action = a->action; p.pi = a->pi; p.latent = a->latent; p.latent_len = a->latent_len; p.sel_steps = a->sel_steps; p.lockstep_levels = a->lockstep_levels;
  p.pow_table = a->pow_table;
  hipError_t e = pl.one ? mzh_launch_one(pl, eng->net, eng->onet, p, (hipStream_t)stream)
                 : pl.wave ? mzh_launch_wave_search(pl, eng->wnet, p, (hipStream_t)stream)
                           : mzh_launch_search(pl, eng->net, p, (hipStream_t)stream);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "search launch");
}

extern "C" int mzh_search(mzh_engine* eng, const mzh_search_args* args, mzh_stream stream) {
  return search_common(eng, args, stream, false);
}

extern "C" int mzh_search_replay(mzh_engine* eng, const mzh_search_args* args, mzh_stream stream) {
  return search_common(eng, args, stream, true);
}

// ---------------------------------------------------------------------------------------------
// fused training update (mzh_train.hip)
namespace {
struct TrainLayout {
  size_t off[22];
  size_t total;  // floats
};
// scratch regions in MztScratch order, each 256-B aligned
TrainLayout train_layout(int B, int U, int support) {
  const size_t BU = (size_t)B * U, ldg = support > 1 ? 48 : 16;
  const size_t sz[] = {(size_t)B * 32, (size_t)B * 256, BU * 64, BU * 256, BU * 256, BU * 256, BU * 256, BU * 64,
                       (size_t)B * 256, (size_t)B * 64, BU * 256, BU * 256, BU * 256, BU * 256, BU * 16, BU * ldg,
                       BU * ldg, BU * 64};
  TrainLayout L{};
  size_t o = 0;
  for (int i = 0; i < 18; ++i) {
    L.off[i] = o;
    o += (sz[i] + 63) & ~(size_t)63;
  }
  L.total = o;
  return L;
}
int train_rows(const mzh_train_args* a) {
  if (a->rows > 0) return a->rows;
  const char* env = getenv("MZH_TRAIN_ROWS");
  if (env) return atoi(env);
  return 1;  // one transition per workgroup: B workgroups (fastest at batch 256, MI355X)
}
}  // namespace

extern "C" int mzh_train_scratch_bytes(int B, int U, int in_dim, int support, size_t* bytes) {
  if (B < 1 || U < 1 || in_dim < 1 || in_dim > 32 || (support != 1 && support != 33) || !bytes)
    return fail(MZH_ERR_ARG, "train_scratch_bytes: bad B=%d U=%d in_dim=%d support=%d", B, U, in_dim, support);
  *bytes = train_layout(B, U, support).total * sizeof(float);
  return MZH_OK;
}

static int train_check(const mzh_train_args* a, bool need_batch) {
  if (!a) return fail(MZH_ERR_ARG, "train: null args");
  if (a->B < 1 || a->U < 1 || a->in_dim < 1 || a->in_dim > 32 || (a->support != 1 && a->support != 33))
    return fail(MZH_ERR_ARG, "train: bad B=%d U=%d in_dim=%d support=%d", a->B, a->U, a->in_dim, a->support);
  for (int i = 0; i < 20; ++i)
    if (!a->param[i] || (need_batch && (!a->exp_avg[i] || !a->exp_avg_sq[i])))
      return fail(MZH_ERR_ARG, "train: null parameter / Adam state pointer %d", i);
  for (int i = 0; i < 10; ++i)
    if (!a->wt[i]) return fail(MZH_ERR_ARG, "train: null transposed weight %d", i);
  if (!need_batch) return MZH_OK;
  if (!a->obs || !a->rwds || !a->actions || !a->pi || !a->returns || !a->row_loss || !a->scratch)
    return fail(MZH_ERR_ARG, "train: null batch / output / scratch pointer");
  if (a->scratch_bytes < train_layout(a->B, a->U, a->support).total * sizeof(float))
    return fail(MZH_ERR_ARG, "train: scratch of %zu bytes is too small", a->scratch_bytes);
  const int R = train_rows(a);
  if (R != 1 && R != 2) return fail(MZH_ERR_ARG, "train: rows must be 1 or 2 (got %d)", R);
  if (R * a->U > 64) return fail(MZH_ERR_ARG, "train: rows * U = %d exceeds 64", R * a->U);
  if (mzt_rows_smem_bytes(R, a->U) > 160 * 1024)
    return fail(MZH_ERR_ARG, "train: U=%d needs %zu B of LDS at rows=%d", a->U, mzt_rows_smem_bytes(R, a->U), R);
  return MZH_OK;
}

// [out, in] of the ten Linear layers in state_dict order (representation layer 1: in = in_dim;
// value / reward layer 2: out = support)
static void layer_dims(const mzh_train_args* a, int l, int* out, int* in) {
  static const int kOut[10] = {256, 64, 256, 64, 256, -1, 256, 6, 256, -1};
  static const int kIn[10] = {-1, 256, 70, 256, 64, 256, 64, 256, 64, 256};
  *out = kOut[l] < 0 ? a->support : kOut[l];
  *in = kIn[l] < 0 ? a->in_dim : kIn[l];
}

extern "C" int mzh_train_transpose(const mzh_train_args* a, mzh_stream stream) {
  int st = train_check(a, false);
  if (st) return st;
  for (int l = 0; l < 10; ++l) {
    int out, in;
    layer_dims(a, l, &out, &in);
    hipError_t e = mzt_launch_transpose(a->param[2 * l], a->wt[l], out, in, (out + 3) & ~3, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "train transpose launch");
  }
  return MZH_OK;
}

extern "C" int mzh_train_update(const mzh_train_args* a, mzh_stream stream) {
  int st = train_check(a, true);
  if (st) return st;
  const int B = a->B, U = a->U, SUP = a->support;
  const TrainLayout lay = train_layout(B, U, SUP);
  float* base = (float*)a->scratch;
  MztScratch s;
  float** regions[] = {&s.x0, &s.repa, &s.h, &s.ap, &s.av, &s.ad, &s.ar, &s.hp, &s.g_rep, &s.g_h0p,
                       &s.g_p, &s.g_v, &s.g_d, &s.g_r, &s.g_lp, &s.g_lv, &s.g_lr, &s.g_hp};
  for (int i = 0; i < 18; ++i) *regions[i] = base + lay.off[i];

  float* const* P = a->param;
  MztRowParams rp;
  rp.B = B;
  rp.U = U;
  rp.in_dim = a->in_dim;
  rp.obs = a->obs;
  rp.rwds = a->rwds;
  rp.pi = a->pi;
  rp.returns = a->returns;
  rp.w = a->weights;
  rp.actions = a->actions;
  rp.row_loss = a->row_loss;
  rp.new_prio = a->new_prio;
  float* const* T = a->wt;
  rp.n = MztNet{P[0],  T[0], P[1],  P[2],  T[1], P[3],  P[4],  T[2], P[5],  P[6],  T[3], P[7],
                P[8],  T[4], P[9],  P[10], T[5], P[11], P[12], T[6], P[13], P[14], T[7], P[15],
                P[16], T[8], P[17], P[18], T[9], P[19]};
  rp.s = s;
  hipError_t e = mzt_launch_rows(train_rows(a), SUP, rp, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(e, "train rows kernel launch");

  const int BU = B * U, ldg = SUP > 1 ? 48 : 16;
  struct Spec {
    const float* X;
    int ldx;
    const float* GY;
    int ldg, M, out, in, onehot;
  };
  const Spec spec[10] = {
      {s.x0, 32, s.g_rep, 256, B, 256, a->in_dim, -1}, {s.repa, 256, s.g_h0p, 64, B, 64, 256, -1},
      {s.h, 64, s.g_d, 256, BU, 256, 70, 64},          {s.ad, 256, s.g_hp, 64, BU, 64, 256, -1},
      {s.hp, 64, s.g_r, 256, BU, 256, 64, -1},         {s.ar, 256, s.g_lr, ldg, BU, SUP, 256, -1},
      {s.h, 64, s.g_p, 256, BU, 256, 64, -1},          {s.ap, 256, s.g_lp, 16, BU, 6, 256, -1},
      {s.h, 64, s.g_v, 256, BU, 256, 64, -1},          {s.av, 256, s.g_lv, ldg, BU, SUP, 256, -1}};
  MztGradParams gp;
  int tiles = 0;
  for (int l = 0; l < 10; ++l) {
    MztGradLayer& L = gp.L[l];
    const Spec& q = spec[l];
    L.X = q.X;
    L.ldx = q.ldx;
    L.GY = q.GY;
    L.ldg = q.ldg;
    L.M = q.M;
    L.out = q.out;
    L.in = q.in;
    L.onehot_from = q.onehot;
    L.nkb = (q.in + 15) / 16;
    L.tile0 = tiles;
    tiles += ((q.out + 15) / 16) * L.nkb;
    L.W = a->param[2 * l];
    L.b = a->param[2 * l + 1];
    L.mW = a->exp_avg[2 * l];
    L.vW = a->exp_avg_sq[2 * l];
    L.mb = a->exp_avg[2 * l + 1];
    L.vb = a->exp_avg_sq[2 * l + 1];
    L.WT = a->wt[l];
    L.ldwt = (q.out + 3) & ~3;
  }
  gp.actions = a->actions;
  gp.step_size = a->step_size;
  gp.bc2_sqrt = a->bc2_sqrt;
  gp.beta1 = a->beta1;
  gp.beta2 = a->beta2;
  gp.eps = a->eps;
  e = mzt_launch_grad_adam(gp, tiles, (hipStream_t)stream);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "train grad/adam kernel launch");
}

extern "C" int mzh_replay_sample(const mzh_replay_args* a, mzh_stream stream) {
  if (!a) return fail(MZH_ERR_ARG, "replay_sample: null args");
  if (a->n < 1 || a->m < 1 || a->m > MZR_MAX_BATCH || a->d_state < 1 || a->U < 1 || a->A < 1)
    return fail(MZH_ERR_ARG, "replay_sample: bad n=%d m=%d (1..%d) d_state=%d U=%d A=%d", a->n, a->m, MZR_MAX_BATCH,
                a->d_state, a->U, a->A);
  if (!a->prio || !a->u || !a->cdf || !a->states || !a->rwds || !a->actions || !a->pi || !a->returns || !a->indx ||
      !a->out_states || !a->out_rwds || !a->out_actions || !a->out_pi || !a->out_returns || !a->status)
    return fail(MZH_ERR_ARG, "replay_sample: null pointer");
  if (reinterpret_cast<uintptr_t>(a->prio) % 16 != 0)
    return fail(MZH_ERR_ARG, "replay_sample: prio must be 16-byte aligned (float4 loads)");
  hipError_t e = mzr_launch_sample(*a, (hipStream_t)stream);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "replay sample launch");
}

extern "C" int mzh_replay_set_priorities(float* prio, int64_t size, const int64_t* indx, const float* values, int m,
                                         int32_t* status, mzh_stream stream) {
  if (!prio || !indx || !values || !status || size < 1 || m < 1)
    return fail(MZH_ERR_ARG, "replay_set_priorities: bad arguments (size=%lld m=%d)", (long long)size, m);
  hipError_t e = mzr_launch_set_priorities(prio, size, indx, values, m, status, (hipStream_t)stream);
  return e == hipSuccess ? MZH_OK : hip_fail(e, "replay set_priorities launch");
}
