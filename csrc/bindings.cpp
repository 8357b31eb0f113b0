// PyTorch operator registration for the gfx950 kernel library: TORCH_LIBRARY(ddlpc, ...)
// declares every operator as torch.ops.ddlpc.<name>; TORCH_LIBRARY_IMPL(ddlpc, CUDA) below
// registers the HIP kernels, and csrc/cpu_ref.cpp registers the C++ reference kernels under
// the CPU key (the dispatcher picks by tensor device).
//
// Tensor conventions: activations are channel-last tensors whose SHAPE is [N, (D,) H, W, C]
// (contiguous), bf16.  Parameters are fp32 in standard PyTorch layouts; packed bf16 weight
// copies are produced by weight_pack.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cstdlib>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "ops.h"

namespace ddlpc {

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be fp32")

const bf16_t* bptr(const at::Tensor& t) { return reinterpret_cast<const bf16_t*>(t.data_ptr()); }
bf16_t* bptr_mut(at::Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }
const float* fptr_opt(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

struct Geo {
  int dims, N, D, H, W, C;
};
Geo geo_of(const at::Tensor& x) {
  TORCH_CHECK(x.dim() == 4 || x.dim() == 5, "expected [N,(D,)H,W,C] channel-last tensor");
  Geo g;
  g.dims = (int)x.dim() - 2;
  g.N = (int)x.size(0);
  g.D = g.dims == 3 ? (int)x.size(1) : 1;
  g.H = (int)x.size(g.dims == 3 ? 2 : 1);
  g.W = (int)x.size(g.dims == 3 ? 3 : 2);
  g.C = (int)x.size(-1);
  return g;
}
std::vector<int64_t> shape_with_c(const Geo& g, int C, int scale = 1) {
  if (g.dims == 2) return {g.N, (int64_t)g.H * scale, (int64_t)g.W * scale, C};
  return {g.N, (int64_t)g.D * scale, (int64_t)g.H * scale, (int64_t)g.W * scale, C};
}

int pow2ceil(int v) { int p = 1; while (p < v) p <<= 1; return p; }

// pixel tile for the 3x3 conv kernels: BM pixels as TD x TH x TW
void conv_tile(int dims, int BM, int W, int& TD, int& TH, int& TW) {
  if (dims == 2) {
    TD = 1;
    TW = W >= 16 ? 16 : 8;
    TH = BM / TW;
  } else {
    TW = W >= 16 ? 16 : 8;
    TH = 4;
    TD = BM / (TW * TH);
  }
}

int pick_bn(int Cout) {
  if (Cout <= 32) return 32;
  if (Cout <= 64) return 64;
  return 128;
}

}  // namespace

// ---- A/B switches for experiments in progress: knob(name, def) = an in-process override
// (torch.ops.ddlpc.set_knob) or else the environment variable DDLPC_<NAME>, or else def.
// Every name a kernel reads is listed in kKnobs; set_knob rejects any other name, so an A/B
// (bench.py --ab, scripts/conv_micro.py --ab) can never silently time two identical
// configurations.  An empty list = no experiment in progress.
namespace {
const char* const kKnobs[] = {""};
bool knob_registered(const std::string& name) {
  for (const char* k : kKnobs)
    if (k[0] != 0 && name == k) return true;
  return false;
}
std::mutex g_knob_mu;
std::unordered_map<std::string, int>& knob_map() {
  static std::unordered_map<std::string, int> m;
  return m;
}
}  // namespace

int knob(const char* name, int def) {
  TORCH_CHECK(knob_registered(name), "knob '", name, "' read but not listed in kKnobs");
  std::lock_guard<std::mutex> lk(g_knob_mu);
  auto& m = knob_map();
  auto it = m.find(name);
  if (it != m.end()) return it->second;
  const std::string env = std::string("DDLPC_") + name;
  const char* e = getenv(env.c_str());
  const int v = e ? atoi(e) : def;
  m.emplace(name, v);                   // (cached: the environment is read once per name)
  return v;
}

namespace {

// in-process knob override -> the previous value (INT64_MIN: never read or set)
int64_t set_knob(const std::string& name, int64_t value) {
  TORCH_CHECK(knob_registered(name), "set_knob: no kernel reads a knob named '", name,
              "' (registered knobs are listed in kKnobs, csrc/bindings.cpp)");
  std::lock_guard<std::mutex> lk(g_knob_mu);
  auto& m = knob_map();
  auto it = m.find(name);
  const int64_t prev = it != m.end() ? it->second : INT64_MIN;
  if (value == INT64_MIN) {             // clear: the next knob() re-reads the environment
    if (it != m.end()) m.erase(it);
  } else {
    m[name] = (int)value;
  }
  return prev;
}

int phys_cus() {
  static int n = -1;
  if (n < 0) {
    hipDeviceProp_t prop;
    int dev = 0;
    hipGetDevice(&dev);
    n = (hipGetDeviceProperties(&prop, dev) == hipSuccess) ? prop.multiProcessorCount : 256;
  }
  return n;
}

// CUs left out of every persistent / chip-filling grid (set_cu_reserve): under data
// parallelism an RCCL kernel launched in the middle of backward needs free workgroup slots
// at once, but the persistent conv / head kernels otherwise hold every CU until they exit
int g_cu_reserve = 0;

// the CU count grids are sized for
int num_cus() { return std::max(8, phys_cus() - g_cu_reserve); }

// fp64 column sums of an fp32 [R][N] partial slab (deterministic two-pass reduction)
at::Tensor reduce_rows(const at::Tensor& partial, int64_t R, int64_t N) {
  auto dopts = partial.options().dtype(at::kDouble);
  at::Tensor sums = at::empty({N}, dopts);
  const int RC = reduce_rows_chunks((int)R);
  at::Tensor tmp = RC > 1 ? at::empty({2 * RC * N}, dopts) : sums;
  reduce_rows_launch(partial.data_ptr<float>(), (int)R, N, tmp.data_ptr<double>(),
                     sums.data_ptr<double>(), cur_stream());
  return sums;
}

// ------------------------------------------------------------------------ conv3 forward
std::vector<at::Tensor> conv3_fwd(const at::Tensor& x1, const c10::optional<at::Tensor>& x2,
                                  const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                                  const c10::optional<at::Tensor>& pscale,
                                  const c10::optional<at::Tensor>& pshift, int64_t cout,
                                  int64_t co1, bool want_stats_in,
                                  const c10::optional<at::Tensor>& pscale2,
                                  const c10::optional<at::Tensor>& pshift2,
                                  const c10::optional<at::Tensor>& bnb_y,
                                  const c10::optional<at::Tensor>& bnb_s4, int64_t groups) {
  CHECK_DEV(x1); CHECK_CONTIG(x1); CHECK_BF16(x1); CHECK_BF16(w); CHECK_CONTIG(w);
  c10::DeviceGuard guard(x1.device());
  const Geo g = geo_of(x1);
  bool want_stats = want_stats_in;
  ConvFwdArgs a{};
  a.dims = g.dims; a.N = g.N; a.D = g.D; a.H = g.H; a.W = g.W;
  a.C1 = g.C;
  a.C2 = 0;
  const bool dual = x2.has_value() && x2->defined();
  if (dual) {
    CHECK_CONTIG(*x2); CHECK_BF16(*x2);
    const Geo g2 = geo_of(*x2);
    TORCH_CHECK(g2.N == g.N && g2.H == g.H && g2.W == g.W && g2.D == g.D, "concat shape mismatch");
    TORCH_CHECK(g.C % 8 == 0 && g2.C % 8 == 0, "concat inputs need C % 8 == 0");
    a.C2 = g2.C;
  }
  a.Cin = a.C1 + a.C2;
  a.taps = g.dims == 2 ? 9 : 27;
  TORCH_CHECK(w.dim() == 3 && w.size(0) == cout && w.size(1) == a.taps && w.size(2) >= a.Cin,
              "packed weight must be [Cout][taps][CinW>=Cin]");
  a.CinW = (int)w.size(2);
  TORCH_CHECK(a.CinW % 8 == 0, "packed weight ci stride must be a multiple of 8");
  a.Cout = (int)cout;
  a.Co1 = co1 > 0 ? (int)co1 : (int)cout;
  TORCH_CHECK(a.Cout % 8 == 0 && a.Co1 % 8 == 0, "Cout and Co1 must be multiples of 8");
  if (pscale.has_value() && pscale->defined()) TORCH_CHECK(a.C1 <= 512, "prologue supports C1 <= 512");
  // BN groups (ConvFwdArgs::groups): group-major statistics rows; pscale / pshift (and the
  // BNB table) per group — pscale / pshift are [groups][C1] views with a common row stride
  // (the scale / shift rows of group statistics [groups][4][C1])
  const bool grouped = groups > 1;
  if (grouped) {
    TORCH_CHECK(groups <= 1024 && g.N % groups == 0, "conv3_fwd: groups must divide the batch");
    TORCH_CHECK(!(pscale2.has_value() && pscale2->defined()), "conv3_fwd groups: no X2 prologue");
    a.groups = (int)groups;
    if (pscale.has_value() && pscale->defined()) {
      TORCH_CHECK(pshift.has_value() && pshift->defined(), "conv3_fwd groups: pscale needs pshift");
      CHECK_F32(*pscale); CHECK_F32(*pshift);
      TORCH_CHECK(pscale->dim() == 2 && pscale->size(0) == groups && pscale->size(1) == g.C &&
                  pscale->stride(1) == 1 && pshift->sizes() == pscale->sizes() &&
                  pshift->strides() == pscale->strides(),
                  "conv3_fwd groups: pscale / pshift must be [groups][C1] views with one row stride");
      a.gstride = pscale->stride(0);
    }
  }
  a.X1 = bptr(x1);
  a.X2 = dual ? bptr(*x2) : nullptr;
  a.pscale = fptr_opt(pscale);
  a.pshift = fptr_opt(pshift);
  a.pscale2 = fptr_opt(pscale2);
  a.pshift2 = fptr_opt(pshift2);
  if (a.pscale2 != nullptr)
    TORCH_CHECK(dual && a.pshift2 != nullptr && a.C1 + a.C2 <= 512 && pscale2->numel() == a.C2,
                "X2 prologue: needs x2, both pscale2/pshift2 [C2], and C1 + C2 <= 512");
  a.Wt = bptr(w);
  a.bias = fptr_opt(bias);
  if (bnb_y.has_value() && bnb_y->defined()) {
    // BN-backward epilogue: the stats rows become that BN's (sum dyh, sum dyh*xhat) partials
    CHECK_CONTIG(*bnb_y); CHECK_BF16(*bnb_y);
    const int64_t ng = grouped ? groups : 1;
    TORCH_CHECK(bnb_s4.has_value() && bnb_s4->defined() && bnb_s4->numel() == ng * 4 * cout,
                "bnb: stats4 [4][Cout] ([groups][4][Cout] with groups) required");
    if (grouped) a.gstride = 4LL * cout;
    CHECK_F32(*bnb_s4); CHECK_CONTIG(*bnb_s4);
    const Geo gy = geo_of(*bnb_y);
    TORCH_CHECK(g.dims == 2 && gy.N == g.N && gy.H == g.H && gy.W == g.W && gy.C == cout,
                "bnb: 2-D, y must have the output's shape");
    TORCH_CHECK(a.Co1 == a.Cout && a.pscale == nullptr && a.pscale2 == nullptr && a.bias == nullptr,
                "bnb: single output, no prologue, no bias");
    a.bnb_y = bptr(*bnb_y);
    a.bnb_s4 = bnb_s4->data_ptr<float>();
    want_stats = true;
  }
  TORCH_CHECK(a.C2 == 0 || a.C1 % 32 == 0, "concat: first input needs C1 % 32 == 0");
  TORCH_CHECK((a.C1 % 8 == 0) && (a.C2 % 8 == 0), "input channels must be multiples of 8 "
              "(the engine pads the 3-channel image to 8)");
  auto opts = x1.options();
  a.npix = (long long)g.N * g.D * g.H * g.W;
  if (g.dims == 3) {
    // the 3-D 32-input-channel layers: depth-streaming resident kernel (conv3x3x3_ds.hip;
    // 32-channel output chunks, outputs split at Co1 for a concat conv's data gradient)
    int grid = 0, smem = 0;
    if (conv3d_ds_plan(a, num_cus(), grid, smem) >= 0) {
      at::Tensor y1 = at::empty(shape_with_c(g, a.Co1), opts);
      at::Tensor y2;
      if (a.Co1 < a.Cout) y2 = at::empty(shape_with_c(g, a.Cout - a.Co1), opts);
      at::Tensor stats;
      if (want_stats) stats = at::empty({(int64_t)grid, 2, a.Cout}, opts.dtype(at::kFloat));
      a.Y1 = bptr_mut(y1);
      a.Y2 = y2.defined() ? bptr_mut(y2) : nullptr;
      a.stats = want_stats ? stats.data_ptr<float>() : nullptr;
      conv3d_ds_launch(a, grid, smem, cur_stream());
      at::Tensor none = at::empty({0}, opts);
      return {y1, y2.defined() ? y2 : none, stats.defined() ? stats : none};
    }
  }
  {
    // high-resolution few-channel layers: resident-weight kernel (conv3x3_res.hip)
    int grid = 0, smem = 0;
    const int variant = conv3_res_plan(a, num_cus(), grid, smem);
    if (variant >= 0) {
      at::Tensor y1 = at::empty(shape_with_c(g, a.Co1), opts);
      at::Tensor y2;
      if (a.Co1 < a.Cout) y2 = at::empty(shape_with_c(g, a.Cout - a.Co1), opts);
      at::Tensor stats;
      if (want_stats) stats = at::empty({(int64_t)grid, 2, a.Cout}, opts.dtype(at::kFloat));
      a.Y1 = bptr_mut(y1);
      a.Y2 = y2.defined() ? bptr_mut(y2) : nullptr;
      a.stats = want_stats ? stats.data_ptr<float>() : nullptr;
      conv3_res_launch(a, variant, grid, smem, cur_stream());
      at::Tensor none = at::empty({0}, opts);
      return {y1, y2.defined() ? y2 : none, stats.defined() ? stats : none};
    }
  }
  // tile configuration: channel tile from Cout, pixel tile from the image size; the
  // 128-channel config drops to a 64-pixel tile when the layer would not fill the chip
  int cfg = a.Cout <= 32 ? 0 : a.Cout <= 64 ? 1 : 2;
  auto plan = [&](int c) {
    const int BM = conv3_fwd_cfg_bm(c);
    conv_tile(g.dims, BM, g.W, a.TD, a.TH, a.TW);
    a.tilesD = (g.D + a.TD - 1) / a.TD;
    a.tilesH = (g.H + a.TH - 1) / a.TH;
    a.tilesW = (g.W + a.TW - 1) / a.TW;
    a.nTilesM = g.N * a.tilesD * a.tilesH * a.tilesW;
    a.nTilesN = (a.Cout + conv3_fwd_cfg_bn(c) - 1) / conv3_fwd_cfg_bn(c);
  };
  plan(cfg);
  if (cfg == 2 && g.dims == 2) {    // 256-pixel tiles on 8 waves if they fill the chip
    plan(4);
    if (a.nTilesM * a.nTilesN >= num_cus()) cfg = 4;
    else plan(cfg);
  }
  // 512-pixel tiles (cfg 5) wherever they fill the chip without padding.  With the rolling
  // fragment pipeline (no scratch spills) every eligible layer gains: 128-input-channel layers
  // 8-10%, K >= 9 x 256 layers 1-2% (same-process A/B at batch 128,
  // profiles/r3s/conv_ab_cfg5_all_r3s7.txt)
  if (cfg == 4 && a.bnb_y == nullptr) {
    plan(5);
    const double w5 = (double)a.nTilesM * 512 / ((double)g.N * g.D * g.H * g.W);
    if (a.nTilesM * a.nTilesN >= num_cus() && w5 <= 1.05) cfg = 5;
    else plan(cfg);
  }
  // 3-D: the 8-wave configurations wherever they fill the chip with little padding (the
  // 4-wave 3-D tiles need so much halo LDS that one workgroup = one wave per SIMD fits a CU)
  if (g.dims == 3 && cfg <= 2) {
    const int c8 = cfg == 0 ? 6 : cfg == 1 ? 7 : a.Cout == 96 ? 9 : 8;
    plan(c8);
    const double w8 = (double)a.nTilesM * conv3_fwd_cfg_bm(c8) / ((double)g.N * g.D * g.H * g.W);
    if (a.nTilesM * a.nTilesN >= num_cus() && w8 <= 1.15 && g.W >= 16) cfg = c8;
    else plan(cfg);
  }
  if (cfg == 2 && a.nTilesM * a.nTilesN < 2 * num_cus()) { cfg = 3; plan(cfg); }
  // small images: a tile larger than the image computes padding (the 8x8 bottleneck layer
  // under a 256-pixel tile is 75% padding: 48.6 -> 32.5 us with 64-pixel tiles, batch 128)
  auto waste = [&](int c) {
    plan(c);
    return (double)a.nTilesM * conv3_fwd_cfg_bm(c) / ((double)g.N * g.D * g.H * g.W);
  };
  while ((cfg == 4 || cfg == 2) && waste(cfg) > 1.3) cfg = cfg == 4 ? 2 : 3;
  if (cfg == 5 && waste(5) > 1.05) cfg = 4;
  if (cfg == 5) { plan(5); TORCH_CHECK(a.TW == 16 && g.dims == 2, "cfg 5: 16-wide 2-D tiles"); }
  plan(cfg);
  TORCH_CHECK((g.dims == 3 ? a.TD + 2 : 1) * (a.TH + 2) * (a.TW + 2) <= conv3_fwd_cfg_halo(g.dims, cfg),
              "halo exceeds LDS capacity");
  // the streaming kernel's epilogue: per-image buffer descriptors (32-bit offsets) and one
  // output per 16-channel tile
  TORCH_CHECK((long long)g.D * g.H * g.W * a.Cout * 4 < (1LL << 31), "conv3: image too large for 32-bit offsets");
  TORCH_CHECK(a.Co1 == a.Cout || a.Co1 % 16 == 0, "split output needs Co1 % 16 == 0");
  at::Tensor y1 = at::empty(shape_with_c(g, a.Co1), opts);
  at::Tensor y2;
  if (a.Co1 < a.Cout) y2 = at::empty(shape_with_c(g, a.Cout - a.Co1), opts);
  at::Tensor stats;
  a.persist_blocks = (cfg >= 4 ? 1 : 2) * num_cus();   // cfg >= 4: one 8-wave workgroup per CU
  // small layers: split the input-channel chunks across workgroups so the grid fills the
  // chip; partial sums go through an fp32 buffer and a deterministic finalize
  const int nchunks_total = (a.Cin + 31) / 32;
  a.ksplit = 1;
  {
    const int items = a.nTilesM * a.nTilesN;
    int best = 1;
    if (items < num_cus() && !grouped)      // (BN groups: group-major rows, no split-K)
      for (int ks = 2; ks <= 8; ++ks)
        if (nchunks_total % ks == 0 && nchunks_total / ks >= 2 && items * ks <= 2 * num_cus())
          best = ks;
    a.ksplit = best;
  }
  at::Tensor part;
  if (a.ksplit > 1) {
    part = at::empty({(int64_t)a.ksplit * a.npix * a.Cout}, opts.dtype(at::kFloat));
    a.part = part.data_ptr<float>();
  }
  // finalize: ~one pixel group per thread (the split-K layers are the small, latency-bound
  // ones: a short grid-stride chain per thread beats fewer, longer-running workgroups)
  const int fin_px_per_block = std::max(1, 256 / (a.Cout / 8));
  const int fin_grid = (int)std::min<long long>(
      std::max<long long>(1, (a.npix + fin_px_per_block - 1) / fin_px_per_block), 2048);
  if (want_stats) {
    const int grid = a.ksplit > 1 ? fin_grid : conv3_fwd_grid(a);
    stats = at::empty({(int64_t)grid, 2, a.Cout}, opts.dtype(at::kFloat));
  }
  a.Y1 = bptr_mut(y1);
  a.Y2 = y2.defined() ? bptr_mut(y2) : nullptr;
  a.stats = want_stats ? stats.data_ptr<float>() : nullptr;
  conv3_fwd_launch(a, cfg, cur_stream());
  if (a.ksplit > 1) conv3_splitk_finalize_launch(a, fin_grid, cur_stream());
  at::Tensor none = at::empty({0}, opts);
  return {y1, y2.defined() ? y2 : none, stats.defined() ? stats : none};
}

// ------------------------------------------------------------------------ conv3 wgrad
at::Tensor conv3_wgrad(const at::Tensor& dy, const at::Tensor& x1,
                       const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& pscale,
                       const c10::optional<at::Tensor>& pshift,
                       const c10::optional<at::Tensor>& out,
                       const c10::optional<at::Tensor>& pscale2,
                       const c10::optional<at::Tensor>& pshift2,
                       const c10::optional<at::Tensor>& dy_y,
                       const c10::optional<at::Tensor>& dy_s4,
                       const c10::optional<at::Tensor>& dy_coefs, int64_t cin_real,
                       int64_t groups, const c10::optional<at::Tensor>& dy_out) {
  CHECK_DEV(dy); CHECK_CONTIG(dy); CHECK_BF16(dy); CHECK_CONTIG(x1); CHECK_BF16(x1);
  c10::DeviceGuard guard(dy.device());
  const Geo g = geo_of(x1);
  const Geo gy = geo_of(dy);
  TORCH_CHECK(gy.N == g.N && gy.H == g.H && gy.W == g.W && gy.D == g.D, "dy/x shape mismatch");
  ConvWgradArgs a{};
  a.dims = g.dims; a.N = g.N; a.D = g.D; a.H = g.H; a.W = g.W;
  a.C1 = g.C; a.C2 = 0;
  const bool dual = x2.has_value() && x2->defined();
  if (dual) { CHECK_CONTIG(*x2); a.C2 = (int)x2->size(-1); }
  a.Cin = a.C1 + a.C2;
  a.Cout = gy.C;
  TORCH_CHECK(a.Cout % 8 == 0, "Cout must be a multiple of 8");
  a.taps = g.dims == 2 ? 9 : 27;
  a.dY = bptr(dy);
  a.X1 = bptr(x1);
  a.X2 = dual ? bptr(*x2) : nullptr;
  a.pscale = fptr_opt(pscale);
  a.pshift = fptr_opt(pshift);
  a.pscale2 = fptr_opt(pscale2);
  a.pshift2 = fptr_opt(pshift2);
  if (a.pscale) TORCH_CHECK(a.C1 <= 512, "prologue supports C1 <= 512");
  // BN groups: the X1 prologue constants per group of images (pscale / pshift: [groups][C1]
  // views with one row stride, as conv3_fwd's); v3 kernel only (checked below)
  if (groups > 1 && a.pscale != nullptr) {
    TORCH_CHECK(groups <= 1024 && g.N % groups == 0, "conv3_wgrad: groups must divide the batch");
    TORCH_CHECK(a.pscale2 == nullptr && !dual, "conv3_wgrad groups: single input, no X2 prologue");
    TORCH_CHECK(pscale->dim() == 2 && pscale->size(0) == groups && pscale->size(1) == a.C1 &&
                pscale->stride(1) == 1 && pshift->sizes() == pscale->sizes() &&
                pshift->strides() == pscale->strides(),
                "conv3_wgrad groups: pscale / pshift must be [groups][C1] views with one row stride");
    a.groups = (int)groups;
    a.gimg = g.N / (int)groups;
    a.gstride = pscale->stride(0);
  }
  if (a.pscale2) TORCH_CHECK(dual && a.pshift2 && a.C1 + a.C2 <= 512, "X2 prologue: x2, pscale2/pshift2, C1 + C2 <= 512");
  int bco = a.Cout <= 32 ? 32 : 64;
  // v2 / v3 (LDS-DMA pixel tiles 16 wide; narrower images run with masked columns: the 8x8
  // bottleneck layers are 10% faster there than on the v1 kernel)
  const bool v2 = g.W >= 8 && (a.C2 == 0 || a.C1 % 32 == 0);
  // v3 (32x32x16 MFMA, conflict-free transposed reads): whole 32-channel input chunks,
  // concat layers included (same-process bench A/B at batch 256: -0.8% step time,
  // profiles/r3s/bench_ab_wgrad3_concat_r3s9.log)
  const bool v3 = v2 && a.C1 % 32 == 0 && a.C2 % 32 == 0;
  const bool emit = dy_out.has_value() && dy_out->defined();
  if (dy_y.has_value() && dy_y->defined()) {
    // dy holds dA; BN backward applied on load: the v2 kernel, or — with dy_out, where the
    // formed dY is also stored — the 32-output-channel concat kernel (checked below)
    CHECK_CONTIG(*dy_y); CHECK_BF16(*dy_y);
    TORCH_CHECK(((v2 && !v3) || emit) && g.dims == 2 && dy_y->numel() == dy.numel(),
                "conv3_wgrad: the dY prologue needs the v2 kernel (2-D, C1 % 32 != 0 or a 32-channel "
                "first layer) or dy_out, and y of dY's shape");
    TORCH_CHECK(dy_s4.has_value() && dy_s4->numel() == 4 * a.Cout && dy_coefs.has_value() &&
                dy_coefs->numel() == 3 * a.Cout, "conv3_wgrad: dy_s4 [4][Cout] and dy_coefs [3][Cout]");
    CHECK_F32(*dy_s4); CHECK_F32(*dy_coefs);
    a.dyy = bptr(*dy_y);
    a.dys4 = dy_s4->data_ptr<float>();
    a.dycoef = dy_coefs->data_ptr<float>();
    if (emit) {
      CHECK_CONTIG(*dy_out); CHECK_BF16(*dy_out);
      TORCH_CHECK(dy_out->numel() == dy.numel(), "conv3_wgrad: dy_out must have dY's shape");
      a.dyout = reinterpret_cast<bf16_t*>(dy_out->data_ptr());
    }
  }
  TORCH_CHECK(!emit || a.dyy != nullptr, "conv3_wgrad: dy_out needs the dY prologue (dy_y, dy_s4, dy_coefs)");
  // the image layer: <= 4 real channels (cin_real, from the caller) of an 8-channel padded
  // input, (tap, channel)-packed kernel
  // (3-D: per depth tap plane, as the v2 / v3 kernels)
  const bool img = cin_real > 0 && cin_real <= 4 && a.C1 == 8 && !dual && g.W >= 16 &&
                   a.pscale == nullptr && a.pscale2 == nullptr;
  // v3 with 128 output channels per workgroup (every wave a 32-channel quarter, no k-split;
  // 96-pixel tiles): each staged input halo feeds twice the MFMAs of the 64-channel tiles
  // (>= 32x32 images: on the 16^2 / 8^2 levels the 96-pixel tiles are mostly masked columns,
  // measured 3-21% slower there)
  if (v3 && !img && a.Cout >= 128 && g.H * g.W >= 32 * 32) bco = 128;
  // v3 with two 32-channel input chunks per 64-output-channel workgroup (each staged dY tile
  // feeds both halos; 96-pixel tiles) on the >= 64x64 layers with >= 2 input chunks: dec2.a
  // -13%, enc2.b / dec2.b -5% in isolation; the 8^2 / 16^2 layers lose 3-23% (masked tile
  // columns): profiles/r3s/wgrad_ab_ciw_b256_r3s21.txt
  a.ciw = 1;
  if (v3 && !img && bco == 64 && a.Cin >= 64 && g.H * g.W >= 64 * 64)
    a.ciw = 2;
  if (img) { a.TD = 1; a.TW = 16; a.TH = conv3_wgrad_img_pt(bco) / 16; }
  else if (v3 && (bco == 128 || a.ciw == 2)) { a.TD = 1; a.TW = 16; a.TH = 6; }
  else if (v3) { a.TD = 1; a.TW = 16; a.TH = bco == 32 ? 16 : 8; }
  else if (v2) { a.TD = 1; a.TW = 16; a.TH = conv3_wgrad2_pt(bco, a.C2, g.H, g.W) / 16; }
  else if (g.dims == 2) { a.TD = 1; a.TW = g.W >= 16 ? 16 : 8; a.TH = 128 / a.TW; }
  else { a.TW = g.W >= 16 ? 16 : 8; a.TH = 4; a.TD = 128 / (a.TW * a.TH); }
  TORCH_CHECK(v2 || (a.TD + (g.dims == 3 ? 2 : 0)) * (a.TH + 2) * (a.TW + 2) <= conv3_wgrad_halo_cap(g.dims),
              "wgrad halo exceeds LDS capacity");
  a.tilesD = (g.D + a.TD - 1) / a.TD;
  a.tilesH = (g.H + a.TH - 1) / a.TH;
  a.tilesW = (g.W + a.TW - 1) / a.TW;
  a.nTiles = g.N * a.tilesD * a.tilesH * a.tilesW;
  a.coTiles = (a.Cout + bco - 1) / bco;
  a.ciChunks = (a.Cin + 32 * a.ciw - 1) / (32 * a.ciw);
  a.planes = g.dims == 2 ? 1 : 3;
  // split-K over pixel tiles: enough blocks to fill the chip, but every block keeps >= 8
  // tiles so the fp32 partial slab stays small next to the MFMA work
  const int base = a.coTiles * a.ciChunks * a.planes;
  // workgroups per CU to aim for: the weight gradient runs concurrently with the data-
  // gradient chain, and its resident workgroups decide what else fits on a CU.  Round 2
  // (other kernels): two, 1 / 3 / 4 -7 / -1.5 / -1.9%; round 5, same box, three interleaved
  // runs each: 1 / 2 / 3 / 4 -> 7508 / 7610-7613 / 7628 / 7611 img/s, window and 3-D within
  // noise (profiles/r5/wgrad_wg_per_cu_g71_g72/): three; re-checked at batch 384 (round 6,
  // bench --ab, two calls): 2 / 4 -> +0.5-0.6% / +0.9-1.0% ms per step (profiles/r6/wgrad_wg_per_cu_b384_r6ac/)
  constexpr int wg_per_cu = 3;
  const int target = wg_per_cu * num_cus();
  int splits = std::max(1, (target + base - 1) / base);
  splits = std::min(splits, std::max(1, a.nTiles / 8));
  a.splits = splits;
  // 3-D, 32 output channels: the depth-streaming kernel (one pass over dY and X for all 27
  // taps) when eligible
  int ds_grid = -1, c32_grid = -1;
  if (g.dims == 3 && !img && a.groups <= 1) {
    ds_grid = conv3d_wgrad_ds_plan(a, num_cus());
    if (ds_grid >= 0) splits = a.splits;
  }
  // 2-D 32-output-channel concat convs: every input chunk per workgroup (dY read once)
  if (g.dims == 2 && !img && a.groups <= 1) {
    c32_grid = conv3_wgrad_c32_plan(a, num_cus());
    if (c32_grid >= 0) splits = a.splits;
  }
  TORCH_CHECK(!emit || c32_grid >= 0, "conv3_wgrad: dy_out only with the 32-output-channel concat "
              "kernel (2-D, Cout 32, 64..96 input channels in 32-channel chunks, W >= 16, no groups)");
  auto part = at::empty({(int64_t)splits * a.Cout * a.taps * a.Cin}, dy.options().dtype(at::kFloat));
  a.partial = part.data_ptr<float>();
  TORCH_CHECK(a.pscale2 == nullptr || v2, "X2 prologue needs the v2/v3 weight-gradient kernels "
              "(2-D or 3-D, W >= 16, C1 % 32 == 0)");
  TORCH_CHECK(a.groups <= 1 || (v3 && !img), "conv3_wgrad groups: the v3 kernel only (W >= 8, C1 % 32 == 0)");
  if (ds_grid >= 0) conv3d_wgrad_ds_launch(a, ds_grid, cur_stream());
  else if (c32_grid >= 0) conv3_wgrad_c32_launch(a, c32_grid, cur_stream());
  else if (img) conv3_wgrad_img_launch(a, bco, cur_stream());
  else if (v3) conv3_wgrad3_launch(a, bco, cur_stream());
  else if (v2) conv3_wgrad2_launch(a, bco, cur_stream());
  else conv3_wgrad_launch(a, bco, cur_stream());
  std::vector<int64_t> wshape = {a.Cout, a.Cin, 3, 3};
  if (g.dims == 3) wshape.push_back(3);
  const bool into = out.has_value() && out->defined();
  if (into) {
    CHECK_F32(*out); CHECK_CONTIG(*out);
    TORCH_CHECK(out->numel() == (int64_t)a.Cout * a.Cin * a.taps, "dW out size mismatch");
  }
  at::Tensor dW = into ? *out : at::empty(wshape, dy.options().dtype(at::kFloat));
  const long long NW = (long long)a.Cout * a.taps * a.Cin;
  at::Tensor tmp = splits > 64 ? at::empty({(int64_t)((splits + 63) / 64) * NW},
                                           dy.options().dtype(at::kDouble))
                               : at::empty({0}, dy.options().dtype(at::kDouble));
  reduce_rows_scatter_launch(part.data_ptr<float>(), splits, NW, tmp.data_ptr<double>(),
                             dW.data_ptr<float>(), 0, a.Cout, a.taps, a.Cin, into, cur_stream());
  return into ? at::empty({0}, dy.options().dtype(at::kFloat)) : dW;
}

// ------------------------------------------------------------------------ fused 32-channel backward
// The second conv of a 32-channel DoubleConv (input relu(bn1(y))): data gradient dA with the
// BN1-backward partial rows [grid][2][32] and the weight gradient (OIHW [32][32][3][3],
// accumulated into dw_out when given) from one pass over dY and y (conv3x3_bwd32.hip)
std::vector<at::Tensor> conv3_bwd32(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& s4,
                                    const at::Tensor& wd, const c10::optional<at::Tensor>& dw_out,
                                    int64_t groups) {
  CHECK_DEV(dy); CHECK_CONTIG(dy); CHECK_BF16(dy); CHECK_CONTIG(y); CHECK_BF16(y);
  CHECK_BF16(wd); CHECK_CONTIG(wd); CHECK_F32(s4); CHECK_CONTIG(s4);
  c10::DeviceGuard guard(dy.device());
  const Geo g = geo_of(dy);
  const Geo gy = geo_of(y);
  TORCH_CHECK(g.dims == 2 && g.C == 32 && gy.dims == 2 && gy.C == 32 && gy.N == g.N && gy.H == g.H &&
              gy.W == g.W, "conv3_bwd32: 2-D dY and y of one shape with 32 channels");
  const int G = groups > 1 ? (int)groups : 1;
  TORCH_CHECK(G <= 1024 && g.N % G == 0, "conv3_bwd32: groups must divide the batch");
  TORCH_CHECK(wd.numel() == 32 * 9 * 32 && s4.numel() == (int64_t)G * 4 * 32,
              "conv3_bwd32: data-gradient pack [32][9][32] and stats4 [4][32] ([groups][4][32])");
  TORCH_CHECK((long long)g.H * g.W * 64 < (1LL << 31), "conv3_bwd32: image too large for 32-bit offsets");
  Bwd32Args a{};
  a.N = g.N; a.H = g.H; a.W = g.W;
  a.dY = bptr(dy); a.Y = bptr(y); a.s4 = s4.data_ptr<float>(); a.Wd = bptr(wd);
  a.tilesH = (g.H + 15) / 16; a.tilesW = (g.W + 15) / 16;
  a.nTiles = g.N * a.tilesH * a.tilesW;
  a.groups = G;
  const int grid = conv3_bwd32_grid(a.nTiles, num_cus(), G);
  auto fopts = dy.options().dtype(at::kFloat);
  at::Tensor dA = at::empty_like(dy);
  at::Tensor bnpart = at::empty({grid, 2, 32}, fopts);
  at::Tensor wpart = at::empty({(int64_t)grid * 32 * 9 * 32}, fopts);
  a.dA = bptr_mut(dA); a.bnpart = bnpart.data_ptr<float>(); a.wpart = wpart.data_ptr<float>();
  conv3_bwd32_launch(a, grid, cur_stream());
  const bool into = dw_out.has_value() && dw_out->defined();
  if (into) {
    CHECK_F32(*dw_out); CHECK_CONTIG(*dw_out);
    TORCH_CHECK(dw_out->numel() == 32 * 32 * 9, "dW out size mismatch");
  }
  at::Tensor dW = into ? *dw_out : at::empty({32, 32, 3, 3}, fopts);
  const long long NW = 32LL * 9 * 32;
  at::Tensor tmp = grid > 64 ? at::empty({(int64_t)((grid + 63) / 64) * NW}, dy.options().dtype(at::kDouble))
                             : at::empty({0}, dy.options().dtype(at::kDouble));
  reduce_rows_scatter_launch(wpart.data_ptr<float>(), grid, NW, tmp.data_ptr<double>(), dW.data_ptr<float>(),
                             0, 32, 9, 32, into, cur_stream());
  return {dA, bnpart, into ? at::empty({0}, fopts) : dW};
}

// ------------------------------------------------------------------------ BatchNorm
// returns stats4 [4][C] = (mean, invstd, scale, shift)
at::Tensor bn_finalize(const at::Tensor& partial, double count, const at::Tensor& gamma,
                       const at::Tensor& beta, at::Tensor running_mean, at::Tensor running_var,
                       double momentum, double eps, bool update_running,
                       const c10::optional<at::Tensor>& nbt) {
  CHECK_F32(partial); CHECK_F32(gamma); CHECK_F32(beta);
  c10::DeviceGuard guard(partial.device());
  const int C = (int)gamma.numel();
  const int P = (int)(partial.numel() / (2 * C));
  at::Tensor st = at::empty({4, C}, partial.options());
  int64_t* nbp = (nbt.has_value() && nbt->defined()) ? nbt->data_ptr<int64_t>() : nullptr;
  if (P <= 4096) {
    bn_stats_finalize_rows_launch(partial.data_ptr<float>(), P, C, count, gamma.data_ptr<float>(),
                                  beta.data_ptr<float>(), running_mean.data_ptr<float>(),
                                  running_var.data_ptr<float>(), (float)momentum, (float)eps,
                                  st.data_ptr<float>(), update_running, nbp, cur_stream());
    return st;
  }
  at::Tensor sums = reduce_rows(partial, P, 2 * C);
  bn_stats_finalize_launch(sums.data_ptr<double>(), C, count, gamma.data_ptr<float>(),
                           beta.data_ptr<float>(), running_mean.data_ptr<float>(),
                           running_var.data_ptr<float>(), (float)momentum, (float)eps,
                           st.data_ptr<float>(), update_running, nbp, cur_stream());
  return st;
}

// deferred BatchNorm running-statistics updates, in micro-batch order (see reduce.hip)
void bn_running_apply(at::Tensor running_mean, at::Tensor running_var, const at::Tensor& slots,
                      double momentum, const c10::optional<at::Tensor>& nbt) {
  // slots: [K][2C] rows of (mean | unbiased var), any row stride (a column slice of a
  // per-micro-batch arena), rows contiguous
  CHECK_F32(running_mean); CHECK_F32(running_var); CHECK_F32(slots);
  const int C = (int)running_mean.numel();
  TORCH_CHECK(running_var.numel() == C && slots.dim() == 2 && slots.size(1) == 2 * C &&
              slots.stride(1) == 1, "slots [K][2C] with contiguous rows");
  c10::DeviceGuard guard(slots.device());
  const int K = (int)slots.size(0);
  if (K == 0) return;
  int64_t* nbp = (nbt.has_value() && nbt->defined()) ? nbt->data_ptr<int64_t>() : nullptr;
  bn_running_apply_launch(running_mean.data_ptr<float>(), running_var.data_ptr<float>(),
                          slots.data_ptr<float>(), K, C, (long long)slots.stride(0), (float)momentum,
                          nbp, cur_stream());
}

// every BatchNorm's deferred running-statistics updates in one launch: entries [L][4] int64
// (running_mean*, running_var*, nbt* | 0, C | arena column << 32), arena rows 0..K-1
void bn_running_apply_all(const at::Tensor& entries, const at::Tensor& arena, int64_t K,
                          int64_t maxC, double momentum) {
  TORCH_CHECK(entries.scalar_type() == at::kLong && entries.is_contiguous() && entries.dim() == 2 &&
              entries.size(1) == 4, "entries [L][4] int64");
  CHECK_F32(arena);
  TORCH_CHECK(arena.dim() == 2 && arena.stride(1) == 1 && arena.size(0) >= K, "arena [rows >= K][cols]");
  c10::DeviceGuard guard(arena.device());
  if (K == 0 || entries.size(0) == 0) return;
  bn_running_apply_all_launch(entries.data_ptr<int64_t>(), (int)entries.size(0), (int)maxC,
                              arena.data_ptr<float>(), (int)K, (long long)arena.stride(0),
                              (float)momentum, cur_stream());
}

std::vector<at::Tensor> bn_relu_apply(const at::Tensor& y, const at::Tensor& stats4, bool pool,
                                      bool full) {
  CHECK_DEV(y); CHECK_CONTIG(y); CHECK_BF16(y);
  c10::DeviceGuard guard(y.device());
  const Geo g = geo_of(y);
  TORCH_CHECK(g.C % 8 == 0, "C must be a multiple of 8");
  const float* s = stats4.data_ptr<float>();
  TORCH_CHECK(full || pool, "bn_relu_apply: full=False only with pool (deferred skip)");
  at::Tensor a = full ? at::empty_like(y) : at::empty({0}, y.options());
  at::Tensor p;
  if (pool) {
    TORCH_CHECK(g.H % 2 == 0 && g.W % 2 == 0 && (g.dims == 2 || g.D % 2 == 0), "pool needs even dims");
    std::vector<int64_t> ps = g.dims == 2 ? std::vector<int64_t>{g.N, g.H / 2, g.W / 2, g.C}
                                          : std::vector<int64_t>{g.N, g.D / 2, g.H / 2, g.W / 2, g.C};
    p = at::empty(ps, y.options());
  }
  bn_relu_apply_launch(bptr(y), s + 2 * g.C, s + 3 * g.C, full ? bptr_mut(a) : nullptr,
                       pool ? bptr_mut(p) : nullptr, g.dims, g.N, g.D, g.H, g.W, g.C, cur_stream());
  return {a, p.defined() ? p : at::empty({0}, y.options())};
}

static bool gscale_is_none(const c10::optional<at::Tensor>& g) { return !(g.has_value() && g->defined()); }

// dY, dgamma, dbeta from dA (+ unpool(dP)) through ReLU and BN
std::vector<at::Tensor> bn_backward(const c10::optional<at::Tensor>& dA,
                                    const c10::optional<at::Tensor>& dP, const at::Tensor& y,
                                    const at::Tensor& stats4, const at::Tensor& gamma,
                                    const c10::optional<at::Tensor>& gscale,
                                    const c10::optional<at::Tensor>& dgamma_out,
                                    const c10::optional<at::Tensor>& dbeta_out,
                                    const c10::optional<at::Tensor>& partial_in) {
  CHECK_DEV(y); CHECK_CONTIG(y); CHECK_BF16(y);
  c10::DeviceGuard guard(y.device());
  const Geo g = geo_of(y);
  const int C = g.C;
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  const bool hasA = dA.has_value() && dA->defined();
  const bool hasP = dP.has_value() && dP->defined();
  TORCH_CHECK(hasA || hasP, "bn_backward needs dA or dP");
  if (hasA) { CHECK_CONTIG(*dA); CHECK_BF16(*dA); }
  if (hasP) { CHECK_CONTIG(*dP); CHECK_BF16(*dP); }
  if (!hasP) TORCH_CHECK(hasA, "dA required without pool");
  const float* s = stats4.data_ptr<float>();
  const float* gs = fptr_opt(gscale);
  const long long items = (long long)g.N * (hasP ? (g.dims == 3 ? g.D / 2 : 1) * (g.H / 2) * (g.W / 2)
                                                 : (long long)g.D * g.H * g.W);
  auto fopts = y.options().dtype(at::kFloat);
  const bf16_t* pA = hasA ? bptr(*dA) : nullptr;
  const bf16_t* pP = hasP ? bptr(*dP) : nullptr;
  // partial_in: (sum dyh, sum dyh*xhat) rows [R][2][C] already produced by the kernel that
  // wrote dA (deferred-BN epilogues); otherwise one reduction pass over dA (+dP) and y
  const bool pre = partial_in.has_value() && partial_in->defined() && partial_in->numel() > 0;
  int nb;
  at::Tensor partial;
  if (pre) {
    TORCH_CHECK(!hasP && gscale_is_none(gscale), "precomputed BN partials: no pool / grad scale");
    CHECK_F32(*partial_in); CHECK_CONTIG(*partial_in);
    TORCH_CHECK(partial_in->numel() % (2 * C) == 0, "partial rows must be [R][2][C]");
    partial = *partial_in;
    nb = (int)(partial.numel() / (2 * C));
  } else {
    nb = bn_bwd_reduce_blocks(items);
    partial = at::empty({nb, 2, C}, fopts);
    bn_bwd_reduce_launch(pA, pP, bptr(y), s + 2 * C, s + 3 * C, s, s + C, gs,
                         partial.data_ptr<float>(), nb, g.dims, g.N, g.D, g.H, g.W, C, cur_stream());
  }
  const bool into = dgamma_out.has_value() && dgamma_out->defined();
  at::Tensor dgamma = into ? *dgamma_out : at::empty({C}, fopts);
  at::Tensor dbeta = into ? *dbeta_out : at::empty({C}, fopts);
  at::Tensor coefs = at::empty({3, C}, fopts);
  const double count = (double)g.N * g.D * g.H * g.W;
  if (nb <= 2048) {
    bn_grad_finalize_rows_launch(partial.data_ptr<float>(), nb, C, count, gamma.data_ptr<float>(),
                                 s + C, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                                 coefs.data_ptr<float>(), into, cur_stream());
  } else {   // many rows (per-tile epilogue partials): coalesced two-pass fp64 reduction
    at::Tensor sums = reduce_rows(partial, nb, 2 * C);
    bn_grad_finalize_launch(sums.data_ptr<double>(), C, count, gamma.data_ptr<float>(), s + C,
                            dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                            coefs.data_ptr<float>(), into, cur_stream());
  }
  at::Tensor dY = at::empty_like(y);
  bn_bwd_apply_launch(pA, pP, bptr(y), s + 2 * C, s + 3 * C, s, s + C, coefs.data_ptr<float>(), gs,
                      bptr_mut(dY), g.dims, g.N, g.D, g.H, g.W, C, cur_stream());
  return {dY, dgamma, dbeta};
}

// BatchNorm backward WITHOUT the apply pass: from precomputed (sum dyh, sum dyh*xhat) rows,
// dgamma / dbeta (accumulated into the outs when given) and the dY coefficients [k|m1|m2]
// for a consumer that applies the backward on load (conv3_wgrad's dY prologue)
std::vector<at::Tensor> bn_grad_coefs(const at::Tensor& partial, const at::Tensor& y,
                                      const at::Tensor& stats4, const at::Tensor& gamma,
                                      const c10::optional<at::Tensor>& dgamma_out,
                                      const c10::optional<at::Tensor>& dbeta_out) {
  CHECK_F32(partial); CHECK_CONTIG(partial); CHECK_F32(gamma);
  c10::DeviceGuard guard(partial.device());
  const Geo g = geo_of(y);
  const int C = g.C;
  TORCH_CHECK(partial.numel() % (2 * C) == 0 && partial.numel() > 0, "partial rows must be [R][2][C]");
  const int nb = (int)(partial.numel() / (2 * C));
  auto fopts = partial.options();
  const bool into = dgamma_out.has_value() && dgamma_out->defined();
  at::Tensor dgamma = into ? *dgamma_out : at::empty({C}, fopts);
  at::Tensor dbeta = into ? *dbeta_out : at::empty({C}, fopts);
  at::Tensor coefs = at::empty({3, C}, fopts);
  const float* s = stats4.data_ptr<float>();
  const double count = (double)g.N * g.D * g.H * g.W;
  if (nb <= 2048) {
    bn_grad_finalize_rows_launch(partial.data_ptr<float>(), nb, C, count, gamma.data_ptr<float>(),
                                 s + C, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                                 coefs.data_ptr<float>(), into, cur_stream());
  } else {
    at::Tensor sums = reduce_rows(partial, nb, 2 * C);
    bn_grad_finalize_launch(sums.data_ptr<double>(), C, count, gamma.data_ptr<float>(), s + C,
                            dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                            coefs.data_ptr<float>(), into, cur_stream());
  }
  return {coefs, dgamma, dbeta};
}

// ------------------------------------------------------------------------ BatchNorm groups
// per-micro-batch statistics groups (Trainer bn_window): y holds `groups` micro-batches one
// after another; -> stats4 [groups][4][C]; with an arena [rows][...] the group's
// (mean | unbiased var) goes to arena row g at column aoff (in-order running-stat update)
at::Tensor bn_group_finalize(const at::Tensor& y, int64_t groups, const at::Tensor& gamma,
                             const at::Tensor& beta, double eps,
                             const c10::optional<at::Tensor>& arena, int64_t aoff) {
  CHECK_DEV(y); CHECK_CONTIG(y); CHECK_BF16(y); CHECK_F32(gamma); CHECK_F32(beta);
  c10::DeviceGuard guard(y.device());
  const Geo g = geo_of(y);
  TORCH_CHECK(groups >= 1 && groups <= 1024 && g.N % groups == 0,
              "bn_group_finalize: 1 <= groups <= 1024 dividing the batch");
  TORCH_CHECK(bn_group_supported(g.dims, false, g.D, g.H, g.W, g.C),
              "bn_group_finalize: C / 8 must be a power of two <= 256");
  const long long gpix = (long long)(g.N / groups) * g.D * g.H * g.W;
  const int nb = bn_group_stats_rows(gpix, g.C, (int)groups);
  auto fopts = y.options().dtype(at::kFloat);
  at::Tensor part = at::empty({groups, nb, 2, g.C}, fopts);
  at::Tensor st = at::empty({groups, 4, g.C}, fopts);
  float* ap = nullptr;
  long long astride = 0;
  if (arena.has_value() && arena->defined()) {
    CHECK_F32(*arena);
    TORCH_CHECK(arena->dim() == 2 && arena->size(0) >= groups && arena->stride(1) == 1 &&
                aoff + 2 * g.C <= arena->size(1), "arena [rows >= groups][>= aoff + 2C]");
    ap = arena->data_ptr<float>() + aoff;
    astride = arena->stride(0);
  }
  bn_group_stats_finalize_launch(bptr(y), (int)groups, gpix, g.C, gamma.data_ptr<float>(),
                                 beta.data_ptr<float>(), (float)eps, st.data_ptr<float>(), ap,
                                 astride, part.data_ptr<float>(), nb, cur_stream());
  return st;
}

// the same statistics from partial rows a conv epilogue wrote group-major (conv3_fwd with
// groups): partial [groups * nb][2][C], count = pixels per group
at::Tensor bn_group_finalize_rows(const at::Tensor& partial, int64_t groups, double count,
                                  const at::Tensor& gamma, const at::Tensor& beta, double eps,
                                  const c10::optional<at::Tensor>& arena, int64_t aoff) {
  CHECK_DEV(partial); CHECK_F32(partial); CHECK_CONTIG(partial); CHECK_F32(gamma); CHECK_F32(beta);
  c10::DeviceGuard guard(partial.device());
  const int64_t C = gamma.numel();
  TORCH_CHECK(groups >= 1 && groups <= 1024 && partial.numel() % (groups * 2 * C) == 0,
              "bn_group_finalize_rows: partial [groups * nb][2][C]");
  const int nb = (int)(partial.numel() / (groups * 2 * C));
  at::Tensor st = at::empty({groups, 4, C}, partial.options());
  float* ap = nullptr;
  long long astride = 0;
  if (arena.has_value() && arena->defined()) {
    CHECK_F32(*arena);
    TORCH_CHECK(arena->dim() == 2 && arena->size(0) >= groups && arena->stride(1) == 1 &&
                aoff + 2 * C <= arena->size(1), "arena [rows >= groups][>= aoff + 2C]");
    ap = arena->data_ptr<float>() + aoff;
    astride = arena->stride(0);
  }
  bn_group_finalize_rows_launch(partial.data_ptr<float>(), nb, (int)groups, (long long)count, (int)C,
                                gamma.data_ptr<float>(), beta.data_ptr<float>(), (float)eps,
                                st.data_ptr<float>(), ap, astride, cur_stream());
  return st;
}

std::vector<at::Tensor> bn_group_apply(const at::Tensor& y, const at::Tensor& stats4,
                                       int64_t groups, bool pool) {
  CHECK_DEV(y); CHECK_CONTIG(y); CHECK_BF16(y); CHECK_F32(stats4); CHECK_CONTIG(stats4);
  c10::DeviceGuard guard(y.device());
  const Geo g = geo_of(y);
  TORCH_CHECK(groups >= 1 && g.N % groups == 0 && stats4.numel() == groups * 4 * g.C,
              "bn_group_apply: stats4 [groups][4][C], groups dividing the batch");
  TORCH_CHECK(g.C % 8 == 0, "C must be a multiple of 8");
  at::Tensor a = at::empty_like(y);
  at::Tensor p;
  if (pool) {
    TORCH_CHECK(g.H % 2 == 0 && g.W % 2 == 0 && (g.dims == 2 || g.D % 2 == 0), "pool needs even dims");
    std::vector<int64_t> ps = g.dims == 2 ? std::vector<int64_t>{g.N, g.H / 2, g.W / 2, g.C}
                                          : std::vector<int64_t>{g.N, g.D / 2, g.H / 2, g.W / 2, g.C};
    p = at::empty(ps, y.options());
  }
  const float* s = stats4.data_ptr<float>();
  bn_relu_apply_launch(bptr(y), s + 2 * g.C, s + 3 * g.C, bptr_mut(a), pool ? bptr_mut(p) : nullptr,
                       g.dims, g.N / (int)groups, g.D, g.H, g.W, g.C, cur_stream(), (int)groups,
                       4LL * g.C);
  return {a, p.defined() ? p : at::empty({0}, y.options())};
}

// dY (+ dgamma, dbeta summed over the groups, accumulated into the outs when given)
std::vector<at::Tensor> bn_group_backward(const c10::optional<at::Tensor>& dA,
                                          const c10::optional<at::Tensor>& dP, const at::Tensor& y,
                                          const at::Tensor& stats4, const at::Tensor& gamma,
                                          int64_t groups,
                                          const c10::optional<at::Tensor>& dgamma_out,
                                          const c10::optional<at::Tensor>& dbeta_out,
                                          const c10::optional<at::Tensor>& partial) {
  CHECK_DEV(y); CHECK_CONTIG(y); CHECK_BF16(y); CHECK_F32(stats4); CHECK_CONTIG(stats4);
  c10::DeviceGuard guard(y.device());
  const Geo g = geo_of(y);
  const int C = g.C;
  const bool hasA = dA.has_value() && dA->defined();
  const bool hasP = dP.has_value() && dP->defined();
  TORCH_CHECK(hasA || hasP, "bn_group_backward needs dA or dP");
  if (hasA) { CHECK_CONTIG(*dA); CHECK_BF16(*dA); TORCH_CHECK(dA->numel() == y.numel(), "dA shape"); }
  if (hasP) { CHECK_CONTIG(*dP); CHECK_BF16(*dP); TORCH_CHECK(dP->numel() * (g.dims == 3 ? 8 : 4) == y.numel(), "dP shape"); }
  TORCH_CHECK(groups >= 1 && groups <= 1024 && g.N % groups == 0 && stats4.numel() == groups * 4 * C,
              "bn_group_backward: stats4 [groups][4][C], 1 <= groups <= 1024 dividing the batch");
  TORCH_CHECK(bn_group_supported(g.dims, hasP, g.D, g.H, g.W, C),
              "bn_group_backward: C / 8 a power of two <= 256, even dims with pool");
  const int Ng = g.N / (int)groups;
  const long long items = (long long)Ng * (hasP ? (g.dims == 3 ? g.D / 2 : 1) * (g.H / 2) * (g.W / 2)
                                                : (long long)g.D * g.H * g.W);
  // partial: group-major rows [groups * nb][2][C] of (sum dyh, sum dyh * xhat) from the
  // data-gradient conv's BN-backward epilogue (conv3_fwd with bnb_y and groups)
  const bool have_part = partial.has_value() && partial->defined();
  if (have_part) {
    CHECK_F32(*partial); CHECK_CONTIG(*partial);
    TORCH_CHECK(!hasP && partial->numel() % (groups * 2 * C) == 0,
                "bn_group_backward: partial [groups * nb][2][C], no pooled gradient");
  }
  const int nb = have_part ? (int)(partial->numel() / (groups * 2 * C)) : bn_group_bwd_rows(items, (int)groups);
  auto fopts = y.options().dtype(at::kFloat);
  at::Tensor part = have_part ? *partial : at::empty({groups, nb, 2, C}, fopts);
  at::Tensor coefs = at::empty({groups, 3, C}, fopts);
  const bool into = dgamma_out.has_value() && dgamma_out->defined();
  at::Tensor dgamma = into ? *dgamma_out : at::empty({C}, fopts);
  at::Tensor dbeta = into ? *dbeta_out : at::empty({C}, fopts);
  at::Tensor dY = at::empty_like(y);
  at::Tensor gsum = at::empty({groups, 2, C}, y.options().dtype(at::kDouble));
  bn_group_backward_launch(hasA ? bptr(*dA) : nullptr, hasP ? bptr(*dP) : nullptr, bptr(y),
                           stats4.data_ptr<float>(), gamma.data_ptr<float>(), dgamma.data_ptr<float>(),
                           dbeta.data_ptr<float>(), into, coefs.data_ptr<float>(),
                           part.data_ptr<float>(), nb, bptr_mut(dY), g.dims, (int)groups, Ng, g.D,
                           g.H, g.W, C, cur_stream(), have_part, gsum.data_ptr<double>());
  return {dY, dgamma, dbeta};
}

static const float* bn4_ptr(const c10::optional<at::Tensor>& bn4, int C) {
  if (!(bn4.has_value() && bn4->defined())) return nullptr;
  CHECK_F32(*bn4); CHECK_CONTIG(*bn4);
  TORCH_CHECK(bn4->numel() == 4 * C, "bn4 must be [4][C] (mean, invstd, scale, shift)");
  TORCH_CHECK(C <= 512, "deferred BatchNorm supports C <= 512");
  return bn4->data_ptr<float>();
}

// ------------------------------------------------------------------------ transposed conv
at::Tensor convt_fwd(const at::Tensor& x, const at::Tensor& wt, const c10::optional<at::Tensor>& bias,
                     int64_t cout, const c10::optional<at::Tensor>& bn4) {
  CHECK_DEV(x); CHECK_CONTIG(x); CHECK_BF16(x); CHECK_BF16(wt);
  c10::DeviceGuard guard(x.device());
  const Geo g = geo_of(x);
  const int S = g.dims == 2 ? 4 : 8;
  TORCH_CHECK(g.C % 8 == 0 && cout % 8 == 0, "channels must be multiples of 8");
  TORCH_CHECK(wt.numel() == (int64_t)S * cout * g.C, "packed convT weight size mismatch");
  GemmArgs a{};
  a.mode = GEMM_CONVT_FWD;
  a.M = g.N * g.D * g.H * g.W;
  a.N = S * (int)cout;
  a.K = g.C;
  a.A = bptr(x);
  a.B = bptr(wt);
  a.bias = fptr_opt(bias);
  a.dims = g.dims; a.Nimg = g.N; a.D = g.D; a.H = g.H; a.W = g.W;
  a.Cin = g.C; a.Cout = (int)cout;
  a.bn4 = bn4_ptr(bn4, g.C);
  TORCH_CHECK((int64_t)a.M * (g.dims == 2 ? 4 : 8) < (int64_t)INT32_MAX, "convT: too many pixels for 32-bit pixel indices");
  at::Tensor out = at::empty(shape_with_c(g, (int)cout, 2), x.options());
  a.C = out.data_ptr();
  if (!convt_res_launch(a, num_cus(), cur_stream())) gemm_launch(a, cur_stream());
  return out;
}

std::vector<at::Tensor> convt_dgrad(const at::Tensor& dout, const at::Tensor& wd, int64_t cin,
                                    const c10::optional<at::Tensor>& bny,
                                    const c10::optional<at::Tensor>& bn4) {
  CHECK_DEV(dout); CHECK_CONTIG(dout); CHECK_BF16(dout); CHECK_BF16(wd);
  c10::DeviceGuard guard(dout.device());
  const Geo go = geo_of(dout);
  Geo g = go;
  g.H /= 2; g.W /= 2; if (g.dims == 3) g.D /= 2;
  const int S = g.dims == 2 ? 4 : 8;
  GemmArgs a{};
  a.mode = GEMM_CONVT_DGRAD;
  a.M = g.N * g.D * g.H * g.W;
  a.N = (int)cin;
  a.K = S * go.C;
  a.A = bptr(dout);
  a.B = bptr(wd);
  a.dims = g.dims; a.Nimg = g.N; a.D = g.D; a.H = g.H; a.W = g.W;
  a.Cin = (int)cin; a.Cout = go.C;
  TORCH_CHECK(go.C % 32 == 0, "convT dgrad needs Cout % 32 == 0");
  TORCH_CHECK((int64_t)a.M * (g.dims == 2 ? 4 : 8) < (int64_t)INT32_MAX, "convT: too many pixels for 32-bit pixel indices");
  at::Tensor dx = at::empty(shape_with_c(g, (int)cin), dout.options());
  a.C = dx.data_ptr();
  at::Tensor bnpart = at::empty({0}, dout.options().dtype(at::kFloat));
  a.bn4 = bn4_ptr(bn4, (int)cin);
  if (a.bn4 != nullptr) {
    TORCH_CHECK(bny.has_value() && bny->defined() && bny->is_contiguous() &&
                bny->numel() == dx.numel() && bny->scalar_type() == at::kBFloat16,
                "convt_dgrad: bny must be the deferred pre-BN input (shape of dx, bf16)");
    a.bny = bptr(*bny);
  }
  const int res_rows = convt_res_rows(a, num_cus());
  if (a.bn4 != nullptr) {
    // one fully written row per workgroup: the resident-weight kernel's persistent
    // workgroups, or the GEMM fallback's tiles (each writes its full-width row, zeros
    // outside its channel tile) — no zero-fill pass
    const long long grid = res_rows > 0 ? res_rows : gemm_nt_grid(a);
    bnpart = at::empty({(int64_t)grid, 2, (int64_t)cin}, dout.options().dtype(at::kFloat));
    a.bnpart = bnpart.data_ptr<float>();
  }
  if (res_rows == 0 || !convt_res_launch(a, num_cus(), cur_stream())) gemm_launch(a, cur_stream());
  return {dx, bnpart};
}

// bias gradient of a transposed conv: per-channel sum of dOut.  When dOut came out of a
// conv3 data-gradient epilogue, its per-workgroup channel sums are already there (rows
// [R][2][Ctot], sum part first): reduce those instead of re-reading dOut.
static at::Tensor convt_bias_grad(const at::Tensor& x, const at::Tensor& dout, const Geo& go,
                                  const c10::optional<at::Tensor>& colsum_rows,
                                  const c10::optional<at::Tensor>& db_out, bool into) {
  auto fopts = x.options().dtype(at::kFloat);
  at::Tensor db = into ? *db_out : at::empty({go.C}, fopts);
  if (colsum_rows.has_value() && colsum_rows->defined() && colsum_rows->numel() > 0) {
    const at::Tensor& cr = *colsum_rows;
    TORCH_CHECK(cr.dim() == 3 && cr.size(1) == 2 && cr.size(2) >= go.C, "colsum rows [R][2][C]");
    const int R = (int)cr.size(0);
    at::Tensor ctmp = R > 64 ? at::empty({(int64_t)((R + 63) / 64) * go.C}, x.options().dtype(at::kDouble))
                             : at::empty({0}, x.options().dtype(at::kDouble));
    reduce_rows_scatter_launch(cr.data_ptr<float>(), R, go.C, ctmp.data_ptr<double>(),
                               db.data_ptr<float>(), 2, 0, 0, 0, into, cur_stream(), 2 * cr.size(2));
  } else {
    const long long P = (long long)go.N * go.D * go.H * go.W;
    const int nb = (int)std::max<long long>(1, std::min<long long>((P + 1023) / 1024, 1024));
    at::Tensor cpart = at::empty({nb, go.C}, fopts);
    channel_sum_launch(bptr(dout), P, go.C, cpart.data_ptr<float>(), nb, cur_stream());
    at::Tensor ctmp = nb > 64 ? at::empty({(int64_t)((nb + 63) / 64) * go.C},
                                          x.options().dtype(at::kDouble))
                              : at::empty({0}, x.options().dtype(at::kDouble));
    reduce_rows_scatter_launch(cpart.data_ptr<float>(), nb, go.C, ctmp.data_ptr<double>(),
                               db.data_ptr<float>(), 2, 0, 0, 0, into, cur_stream());
  }
  return db;
}

// Fused data + weight gradient of a 2-D 64 -> 64-channel transposed conv (dOut read once):
// returns {dx, bnpart (deferred BN of x: [R][2][64] rows, else empty), dW, db} (dW / db
// accumulated into the outs when given, empty then).  Other shapes: the separate kernels.
std::vector<at::Tensor> convt_wgrad(const at::Tensor& x, const at::Tensor& dout,
                                    const c10::optional<at::Tensor>& dw_out,
                                    const c10::optional<at::Tensor>& db_out,
                                    const c10::optional<at::Tensor>& colsum_rows,
                                    const c10::optional<at::Tensor>& bn4);

bool convt_bwd_fused_ok(const at::Tensor& x, const at::Tensor& dout) {
  if (x.dim() != 4 || dout.dim() != 4 || x.size(3) != 64 || dout.size(3) != 64) return false;
  if (dout.size(1) != 2 * x.size(1) || dout.size(2) != 2 * x.size(2)) return false;
  const long long K = x.size(0) * x.size(1) * x.size(2);
  if (K * 4 >= (long long)INT32_MAX) return false;
  // one buffer descriptor per split over its dOut rows (32-bit offsets)
  const long long splits = std::max<long long>(1, std::min<long long>(2LL * num_cus(), K / 128));
  const long long per = (K + splits - 1) / splits + 64;
  return (4 * per + 8LL * x.size(2)) * 64 * 2 < (1LL << 31);
}

std::vector<at::Tensor> convt_bwd_fused(const at::Tensor& x, const at::Tensor& dout, const at::Tensor& wd,
                                        const c10::optional<at::Tensor>& dw_out,
                                        const c10::optional<at::Tensor>& db_out,
                                        const c10::optional<at::Tensor>& colsum_rows,
                                        const c10::optional<at::Tensor>& bn4) {
  CHECK_DEV(x); CHECK_CONTIG(x); CHECK_BF16(x); CHECK_CONTIG(dout); CHECK_BF16(dout);
  CHECK_BF16(wd); CHECK_CONTIG(wd);
  c10::DeviceGuard guard(x.device());
  const bool into = dw_out.has_value() && dw_out->defined();
  auto fopts = x.options().dtype(at::kFloat);
  if (!convt_bwd_fused_ok(x, dout)) {
    const bool has_bn = bn4.has_value() && bn4->defined();
    auto r = convt_dgrad(dout, wd, x.size(3), has_bn ? c10::optional<at::Tensor>(x) : c10::nullopt, bn4);
    auto w = convt_wgrad(x, dout, dw_out, db_out, colsum_rows, bn4);
    return {r[0], r[1], w[0], w[1]};
  }
  TORCH_CHECK(wd.numel() == 64 * 256, "convt_bwd_fused: packed dgrad weights must be [64][256]");
  const Geo g = geo_of(x);
  const Geo go = geo_of(dout);
  GemmArgs a{};
  a.mode = GEMM_CONVT_WGRAD;
  a.M = 64; a.N = 256;
  a.K = g.N * g.H * g.W;
  a.A = bptr(x);
  a.B = bptr(dout);
  a.Wd2 = bptr(wd);
  a.dims = 2; a.Nimg = g.N; a.D = 1; a.H = g.H; a.W = g.W;
  a.Cin = 64; a.Cout = 64;
  a.bn4 = bn4_ptr(bn4, 64);
  a.splits = convt_bwd_fused_splits(a.K, num_cus());
  at::Tensor dx = at::empty_like(x);
  a.C = dx.data_ptr();
  at::Tensor part = at::empty({(int64_t)a.splits * 64 * 256}, fopts);
  a.partial = part.data_ptr<float>();
  at::Tensor bnpart = at::empty({a.bn4 != nullptr ? (int64_t)a.splits : 0, 2, 64}, fopts);
  if (a.bn4 != nullptr) a.bnpart = bnpart.data_ptr<float>();
  convt_bwd_fused_launch(a, cur_stream());
  at::Tensor dW = into ? *dw_out : at::empty({64, 64, 2, 2}, fopts);
  const long long NW = 64LL * 256;
  at::Tensor tmp = a.splits > 64 ? at::empty({(int64_t)((a.splits + 63) / 64) * NW}, x.options().dtype(at::kDouble))
                                 : at::empty({0}, x.options().dtype(at::kDouble));
  reduce_rows_scatter_launch(part.data_ptr<float>(), a.splits, NW, tmp.data_ptr<double>(),
                             dW.data_ptr<float>(), 1, 64, 4, 64, into, cur_stream());
  at::Tensor db = convt_bias_grad(x, dout, go, colsum_rows, db_out, into);
  if (into) return {dx, bnpart, at::empty({0}, fopts), at::empty({0}, fopts)};
  return {dx, bnpart, dW, db};
}

std::vector<at::Tensor> convt_wgrad(const at::Tensor& x, const at::Tensor& dout,
                                    const c10::optional<at::Tensor>& dw_out,
                                    const c10::optional<at::Tensor>& db_out,
                                    const c10::optional<at::Tensor>& colsum_rows,
                                    const c10::optional<at::Tensor>& bn4) {
  CHECK_DEV(x); CHECK_CONTIG(x); CHECK_CONTIG(dout);
  c10::DeviceGuard guard(x.device());
  const Geo g = geo_of(x);
  const Geo go = geo_of(dout);
  const int S = g.dims == 2 ? 4 : 8;
  GemmArgs a{};
  a.mode = GEMM_CONVT_WGRAD;
  a.M = g.C;
  a.N = S * go.C;
  a.K = g.N * g.D * g.H * g.W;
  a.A = bptr(x);
  a.B = bptr(dout);
  a.dims = g.dims; a.Nimg = g.N; a.D = g.D; a.H = g.H; a.W = g.W;
  a.Cin = g.C; a.Cout = go.C;
  a.bn4 = bn4_ptr(bn4, g.C);
  // v2 kernel (64 x 64 wave tiles, LDS-DMA stages): enough 128 x 128 workgroups for two per
  // CU, every split >= 4 stages of 64 pixels (other shapes: the v1 kernel)
  int splits;
  a.wg2 = g.C % 8 == 0 && go.C % 8 == 0 && g.C <= 512;
  if (a.wg2) {
    const int tiles = convt_wgrad2_tiles(a);
    splits = std::max(1, (2 * num_cus() + tiles - 1) / tiles);
    splits = std::min(splits, std::max(1, a.K / 256));
    // the kernel addresses a split's dOut rows through one buffer descriptor (32-bit
    // offsets): bound the rows a split can span (up to 2 extra input rows / planes)
    const long long per = ((long long)a.K + splits - 1) / splits + 64;
    const long long span = g.dims == 2 ? 4 * per + 8LL * g.W : 8 * per + 16LL * g.H * g.W;
    if (span * go.C * 2 >= (1LL << 31)) a.wg2 = 0;
  }
  if (!a.wg2) {
    const int base = ((a.M + 63) / 64) * ((a.N + 63) / 64);
    splits = std::max(1, (4 * num_cus() + base - 1) / base);
    splits = std::min(splits, std::max(1, a.K / 256));
  }
  a.splits = splits;
  auto fopts = x.options().dtype(at::kFloat);
  at::Tensor part = at::empty({(int64_t)splits * a.M * a.N}, fopts);
  a.partial = part.data_ptr<float>();
  gemm_launch(a, cur_stream());
  std::vector<int64_t> ws = {g.C, go.C, 2, 2};
  if (g.dims == 3) ws.push_back(2);
  const bool into = dw_out.has_value() && dw_out->defined();
  at::Tensor dW = into ? *dw_out : at::empty(ws, fopts);
  const long long NW = (long long)a.M * a.N;
  at::Tensor tmp = splits > 64 ? at::empty({(int64_t)((splits + 63) / 64) * NW},
                                           x.options().dtype(at::kDouble))
                               : at::empty({0}, x.options().dtype(at::kDouble));
  reduce_rows_scatter_launch(part.data_ptr<float>(), splits, NW, tmp.data_ptr<double>(),
                             dW.data_ptr<float>(), 1, g.C, S, go.C, into, cur_stream());
  at::Tensor db = convt_bias_grad(x, dout, go, colsum_rows, db_out, into);
  if (into) return {at::empty({0}, fopts), at::empty({0}, fopts)};
  return {dW, db};
}

// ------------------------------------------------------------------------ head + CE
at::Tensor head_ce_fwd(const at::Tensor& a, const at::Tensor& Wh, const at::Tensor& bh,
                       const at::Tensor& labels, int64_t ignore_index,
                       const c10::optional<at::Tensor>& bn4) {
  CHECK_DEV(a); CHECK_CONTIG(a); CHECK_BF16(a); CHECK_F32(Wh); CHECK_CONTIG(Wh);
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous(), "labels must be int64");
  c10::DeviceGuard guard(a.device());
  const int C = (int)a.size(-1), K = (int)Wh.size(0);
  TORCH_CHECK(head_supported(C, K), "head kernel: unsupported (C, K)");
  const long long P = a.numel() / C;
  TORCH_CHECK(labels.numel() == P, "labels size mismatch");
  const int nb = (int)std::max<long long>(1, std::min<long long>((P + 255) / 256, 2048));
  auto fopts = a.options().dtype(at::kFloat);
  at::Tensor partial = at::empty({nb, 3}, fopts);
  at::Tensor out3 = at::empty({3}, fopts);
  head_ce_fwd_launch(bptr(a), Wh.data_ptr<float>(), bh.data_ptr<float>(), labels.data_ptr<int64_t>(),
                     partial.data_ptr<float>(), out3.data_ptr<float>(), bn4_ptr(bn4, C), nb, P, C, K,
                     (int)ignore_index, cur_stream());
  return out3;
}

std::vector<at::Tensor> head_ce_bwd(const at::Tensor& a, const at::Tensor& Wh, const at::Tensor& bh,
                                    const at::Tensor& labels, const at::Tensor& out3,
                                    const c10::optional<at::Tensor>& gscale, int64_t ignore_index,
                                    const c10::optional<at::Tensor>& dw_out,
                                    const c10::optional<at::Tensor>& db_out,
                                    const c10::optional<at::Tensor>& bn4, bool store_da) {
  CHECK_DEV(a); CHECK_CONTIG(a);
  c10::DeviceGuard guard(a.device());
  const int C = (int)a.size(-1), K = (int)Wh.size(0);
  const float* pbn = bn4_ptr(bn4, C);
  TORCH_CHECK(head_supported(C, K), "head kernel: unsupported (C, K)");
  TORCH_CHECK(store_da || pbn != nullptr, "head_ce_bwd: store_da=False needs the deferred BN (bn4)");
  const long long P = a.numel() / C;
  const int nb = head_ce_bwd_blocks(C, K, pbn != nullptr, P, num_cus());
  auto fopts = a.options().dtype(at::kFloat);
  // store_da=False: the stats pass of the two-pass backward (head_ce_bn_bwd writes dY)
  at::Tensor dA = store_da ? at::empty_like(a) : at::empty({0}, a.options());
  at::Tensor part = at::empty({nb, K * C + K}, fopts);
  // deferred BatchNorm input: the kernel also emits that BN's backward partial rows
  at::Tensor bnpart = pbn != nullptr ? at::empty({nb, 2, C}, fopts) : at::empty({0}, fopts);
  head_ce_bwd_launch(bptr(a), Wh.data_ptr<float>(), bh.data_ptr<float>(), labels.data_ptr<int64_t>(),
                     fptr_opt(gscale), out3.data_ptr<float>(), 0, store_da ? bptr_mut(dA) : nullptr,
                     part.data_ptr<float>(), nb, P, C, K, (int)ignore_index, pbn,
                     pbn != nullptr ? bnpart.data_ptr<float>() : nullptr, cur_stream());
  const bool into = dw_out.has_value() && dw_out->defined();
  at::Tensor sums = reduce_rows(part, nb, K * C + K);   // rows are [dW (K*C) | db (K)]
  if (into) {
    TORCH_CHECK(dw_out->is_contiguous() && db_out->is_contiguous(), "grad outs must be contiguous");
    scatter_sums_launch(sums.data_ptr<double>(), K * C, dw_out->data_ptr<float>(), 2, 0, 0, 0, 1.f,
                        true, cur_stream());
    scatter_sums_launch(sums.data_ptr<double>() + K * C, K, db_out->data_ptr<float>(), 2, 0, 0, 0,
                        1.f, true, cur_stream());
    at::Tensor none = at::empty({0}, fopts);
    return {dA, none, none, bnpart};
  }
  at::Tensor red = at::empty({K * C + K}, fopts);
  scatter_sums_launch(sums.data_ptr<double>(), K * C + K, red.data_ptr<float>(), 2, 0, 0, 0, 1.f,
                      false, cur_stream());
  at::Tensor dW = red.narrow(0, 0, K * C).view({K, C});
  at::Tensor db = red.narrow(0, K * C, K);
  return {dA, dW, db, bnpart};
}

// Second pass of the two-pass head backward: the last decoder block's BatchNorm backward
// applied to the recomputed head gradient.  partial: the stats pass's [R][2][C] rows;
// returns {dY, dgamma, dbeta} like bn_backward (accumulated into the outs when given)
std::vector<at::Tensor> head_ce_bn_bwd(const at::Tensor& a, const at::Tensor& Wh, const at::Tensor& bh,
                                       const at::Tensor& labels, const at::Tensor& out3,
                                       const c10::optional<at::Tensor>& gscale, int64_t ignore_index,
                                       const at::Tensor& bn4, const at::Tensor& partial,
                                       const at::Tensor& gamma,
                                       const c10::optional<at::Tensor>& dgamma_out,
                                       const c10::optional<at::Tensor>& dbeta_out,
                                       const c10::optional<at::Tensor>& pscale, int64_t groups) {
  CHECK_DEV(a); CHECK_CONTIG(a); CHECK_BF16(a);
  // pscale: device factor on the partial rows (rows from the fused forward at unit scale)
  const float* ps = fptr_opt(pscale);
  c10::DeviceGuard guard(a.device());
  const int C = (int)a.size(-1), K = (int)Wh.size(0);
  if (groups > 1) {
    // BN groups (a batched window): bn4 [groups][4][C], partial rows group-major (the fused
    // forward's head_ce_fwd_stats with groups), per-group coefficients
    const long long P = a.numel() / C;
    TORCH_CHECK(C == 32 && K <= 16 && P % (groups * 16) == 0,
                "head_ce_bn_bwd groups: C = 32 head, pixels per group a multiple of 16");
    CHECK_F32(bn4); CHECK_CONTIG(bn4); CHECK_F32(partial); CHECK_CONTIG(partial); CHECK_F32(gamma);
    TORCH_CHECK(bn4.numel() == groups * 4 * C && partial.numel() % (groups * 2 * C) == 0,
                "head_ce_bn_bwd groups: bn4 [groups][4][C], partial [groups * R][2][C]");
    auto fopts = a.options().dtype(at::kFloat);
    const bool into = dgamma_out.has_value() && dgamma_out->defined();
    at::Tensor dgamma = into ? *dgamma_out : at::empty({C}, fopts);
    at::Tensor dbeta = into ? *dbeta_out : at::empty({C}, fopts);
    at::Tensor coefs = at::empty({groups, 3, C}, fopts);
    at::Tensor gsum = at::empty({groups, 2, C}, a.options().dtype(at::kDouble));
    const int nb = (int)(partial.numel() / (groups * 2 * C));
    bn_group_grad_rows_launch(partial.data_ptr<float>(), nb, (int)groups, C, (double)(P / groups),
                              gamma.data_ptr<float>(), bn4.data_ptr<float>(), dgamma.data_ptr<float>(),
                              dbeta.data_ptr<float>(), into, coefs.data_ptr<float>(),
                              gsum.data_ptr<double>(), ps, cur_stream());
    at::Tensor dY = at::empty_like(a);
    head_bn_apply_launch(bptr(a), Wh.data_ptr<float>(), bh.data_ptr<float>(), labels.data_ptr<int64_t>(),
                         fptr_opt(gscale), out3.data_ptr<float>(), bn4.data_ptr<float>(),
                         coefs.data_ptr<float>(), bptr_mut(dY), P, C, K, (int)ignore_index, cur_stream(),
                         (int)groups);
    return {dY, dgamma, dbeta};
  }
  const float* pbn = bn4_ptr(bn4, C);
  TORCH_CHECK(head_supported(C, K), "head kernel: unsupported (C, K)");
  CHECK_F32(partial); CHECK_CONTIG(partial); CHECK_F32(gamma);
  TORCH_CHECK(partial.numel() % (2 * C) == 0 && partial.numel() > 0, "partial rows must be [R][2][C]");
  const long long P = a.numel() / C;
  const int nb = (int)(partial.numel() / (2 * C));
  auto fopts = a.options().dtype(at::kFloat);
  const bool into = dgamma_out.has_value() && dgamma_out->defined();
  at::Tensor dgamma = into ? *dgamma_out : at::empty({C}, fopts);
  at::Tensor dbeta = into ? *dbeta_out : at::empty({C}, fopts);
  at::Tensor coefs = at::empty({3, C}, fopts);
  const float* s = pbn;
  if (nb <= 2048) {
    bn_grad_finalize_rows_launch(partial.data_ptr<float>(), nb, C, (double)P, gamma.data_ptr<float>(),
                                 s + C, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                                 coefs.data_ptr<float>(), into, cur_stream(), ps);
  } else {
    at::Tensor sums = reduce_rows(partial, nb, 2 * C);
    bn_grad_finalize_launch(sums.data_ptr<double>(), C, (double)P, gamma.data_ptr<float>(), s + C,
                            dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
                            coefs.data_ptr<float>(), into, cur_stream(), ps);
  }
  at::Tensor dY = at::empty_like(a);
  head_bn_apply_launch(bptr(a), Wh.data_ptr<float>(), bh.data_ptr<float>(), labels.data_ptr<int64_t>(),
                       fptr_opt(gscale), out3.data_ptr<float>(), pbn, coefs.data_ptr<float>(),
                       bptr_mut(dY), P, C, K, (int)ignore_index, cur_stream());
  return {dY, dgamma, dbeta};
}

// Training forward of the head with the deferred BatchNorm, fused with the backward's
// statistics pass at a unit gradient scale: returns {out3 = (loss, correct, count),
// dW rows [R][K*C + K], BN partial rows [R][2][C]}.  The backward scales the reductions by
// dL/count on the device (head_wgrad_from_rows, head_ce_bn_bwd pscale).
std::vector<at::Tensor> head_ce_fwd_stats(const at::Tensor& a, const at::Tensor& Wh,
                                          const at::Tensor& bh, const at::Tensor& labels,
                                          int64_t ignore_index, const at::Tensor& bn4,
                                          int64_t groups) {
  CHECK_DEV(a); CHECK_CONTIG(a); CHECK_BF16(a); CHECK_CONTIG(labels);
  TORCH_CHECK(labels.scalar_type() == at::kLong, "labels must be int64");
  c10::DeviceGuard guard(a.device());
  const int C = (int)a.size(-1), K = (int)Wh.size(0);
  const long long P = a.numel() / C;
  const float* pbn = nullptr;
  if (groups > 1) {
    // BN groups: per-group statistics bn4 [groups][4][C], group-major rows (C = 32 kernel)
    CHECK_F32(bn4); CHECK_CONTIG(bn4);
    TORCH_CHECK(C == 32 && K <= 16 && P % (groups * 16) == 0 && bn4.numel() == groups * 4 * C,
                "head_ce_fwd_stats groups: C = 32 head, bn4 [groups][4][C], pixels per group a "
                "multiple of 16");
    pbn = bn4.data_ptr<float>();
  } else {
    pbn = bn4_ptr(bn4, C);
  }
  TORCH_CHECK(head_supported(C, K), "head kernel: unsupported (C, K)");
  TORCH_CHECK(labels.numel() == P, "labels / activation pixel count mismatch");
  const int nb = head_fwd_stats_blocks(C, K, P, num_cus(), groups > 1 ? (int)groups : 1);
  auto fopts = a.options().dtype(at::kFloat);
  at::Tensor wrows = at::empty({nb, K * C + K}, fopts);
  at::Tensor brows = at::empty({nb, 2, C}, fopts);
  at::Tensor lrows = at::empty({nb, 3}, fopts);
  at::Tensor out3 = at::empty({3}, fopts);
  head_ce_fwd_stats_launch(bptr(a), Wh.data_ptr<float>(), bh.data_ptr<float>(), labels.data_ptr<int64_t>(),
                           pbn, wrows.data_ptr<float>(), brows.data_ptr<float>(), lrows.data_ptr<float>(),
                           out3.data_ptr<float>(), nb, P, C, K, (int)ignore_index, cur_stream(),
                           groups > 1 ? (int)groups : 1);
  return {out3, wrows, brows};
}

// dWh, dbh from the fused forward's rows: deterministic fp64 row sums times a device scale
std::vector<at::Tensor> head_wgrad_from_rows(const at::Tensor& rows, const at::Tensor& scale, int64_t K,
                                             int64_t C, const c10::optional<at::Tensor>& dw_out,
                                             const c10::optional<at::Tensor>& db_out) {
  CHECK_F32(rows); CHECK_CONTIG(rows); CHECK_F32(scale);
  c10::DeviceGuard guard(rows.device());
  TORCH_CHECK(rows.dim() == 2 && rows.size(1) == K * C + K, "rows must be [R][K*C + K]");
  const int R = (int)rows.size(0);
  at::Tensor sums = reduce_rows(rows, R, K * C + K);
  auto fopts = rows.options();
  const bool into = dw_out.has_value() && dw_out->defined();
  if (into) {
    TORCH_CHECK(dw_out->is_contiguous() && db_out->is_contiguous(), "grad outs must be contiguous");
    if (db_out->data_ptr<float>() == dw_out->data_ptr<float>() + K * C) {
      // adjacent in the flat gradient buffer (weight then bias): one launch
      scatter_sums_dscale_launch(sums.data_ptr<double>(), K * C + K, dw_out->data_ptr<float>(),
                                 scale.data_ptr<float>(), true, cur_stream());
    } else {
      scatter_sums_dscale_launch(sums.data_ptr<double>(), K * C, dw_out->data_ptr<float>(),
                                 scale.data_ptr<float>(), true, cur_stream());
      scatter_sums_dscale_launch(sums.data_ptr<double>() + K * C, K, db_out->data_ptr<float>(),
                                 scale.data_ptr<float>(), true, cur_stream());
    }
    return {at::empty({0}, fopts), at::empty({0}, fopts)};
  }
  at::Tensor red = at::empty({K * C + K}, fopts);
  scatter_sums_dscale_launch(sums.data_ptr<double>(), K * C + K, red.data_ptr<float>(),
                             scale.data_ptr<float>(), false, cur_stream());
  return {red.narrow(0, 0, K * C).view({K, C}), red.narrow(0, K * C, K)};
}

// dL/count as a device scalar from the loss kernel's out3 = (loss, correct, count) and the
// incoming dL (absent: 1)
at::Tensor head_grad_scale(const at::Tensor& out3, const c10::optional<at::Tensor>& gs) {
  CHECK_F32(out3); CHECK_CONTIG(out3);
  TORCH_CHECK(out3.numel() >= 3, "out3 must hold (loss, correct, count)");
  c10::DeviceGuard guard(out3.device());
  const float* pg = nullptr;
  if (gs.has_value() && gs->defined()) {
    CHECK_F32(*gs); CHECK_CONTIG(*gs);
    TORCH_CHECK(gs->numel() == 1 && gs->device() == out3.device(), "gs must be one float on out3's device");
    pg = gs->data_ptr<float>();
  }
  at::Tensor scale = at::empty({1}, out3.options());
  head_grad_scale_launch(out3.data_ptr<float>(), pg, scale.data_ptr<float>(), cur_stream());
  return scale;
}

// DeviceMeter accumulation in one launch (buf: 4 doubles; loss / correct: one float each)
void meter_add(at::Tensor& buf, const at::Tensor& loss, const at::Tensor& correct, double pixels,
               double count) {
  TORCH_CHECK(buf.scalar_type() == at::kDouble && buf.numel() == 4 && buf.is_contiguous(),
              "meter buffer must be 4 contiguous doubles");
  CHECK_F32(loss); CHECK_F32(correct);
  TORCH_CHECK(loss.numel() == 1 && correct.numel() == 1, "loss / correct must be scalars");
  TORCH_CHECK(loss.device() == buf.device() && correct.device() == buf.device(), "device mismatch");
  c10::DeviceGuard guard(buf.device());
  meter_add_launch(buf.data_ptr<double>(), loss.data_ptr<float>(), correct.data_ptr<float>(), pixels,
                   count, cur_stream());
}

at::Tensor head_logits(const at::Tensor& a, const at::Tensor& Wh, const at::Tensor& bh,
                       const c10::optional<at::Tensor>& bn4) {
  CHECK_DEV(a); CHECK_CONTIG(a);
  c10::DeviceGuard guard(a.device());
  const Geo g = geo_of(a);
  const int C = g.C, K = (int)Wh.size(0);
  TORCH_CHECK(head_supported(C, K), "head kernel: unsupported (C, K)");
  const long long HW = (long long)g.D * g.H * g.W;
  std::vector<int64_t> os = g.dims == 2 ? std::vector<int64_t>{g.N, K, g.H, g.W}
                                        : std::vector<int64_t>{g.N, K, g.D, g.H, g.W};
  at::Tensor out = at::empty(os, a.options().dtype(at::kFloat));
  head_logits_launch(bptr(a), Wh.data_ptr<float>(), bh.data_ptr<float>(), out.data_ptr<float>(),
                     (long long)g.N * HW, HW, C, K, bn4_ptr(bn4, C), cur_stream());
  return out;
}

// ------------------------------------------------------------------------ optimizer / pack
void adam_step(at::Tensor p, const at::Tensor& g, at::Tensor m, at::Tensor v, double b1, double b2,
               double eps, double wd, double step_size, double inv_sqrt_bc2) {
  CHECK_DEV(p); CHECK_F32(p); CHECK_F32(g); CHECK_F32(m); CHECK_F32(v);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "size");
  c10::DeviceGuard guard(p.device());
  adam_launch(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
              p.numel(), (float)b1, (float)b2, (float)eps, (float)wd, (float)step_size,
              (float)inv_sqrt_bc2, cur_stream());
}

// graph-capturable step: scal = device float[3] (t, step_size, inv_sqrt_bc2), advanced on
// the device by this call
void adam_step_dev(at::Tensor p, const at::Tensor& g, at::Tensor m, at::Tensor v, at::Tensor scal,
                   double lr, double b1, double b2, double eps, double wd) {
  CHECK_DEV(p); CHECK_F32(p); CHECK_F32(g); CHECK_F32(m); CHECK_F32(v); CHECK_F32(scal);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "size");
  TORCH_CHECK(scal.numel() >= 3 && scal.is_contiguous(), "scal must be float[3]");
  c10::DeviceGuard guard(p.device());
  adam_scalars_launch(scal.data_ptr<float>(), lr, b1, b2, cur_stream());
  adam_launch(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
              p.numel(), (float)b1, (float)b2, (float)eps, (float)wd, 0.f, 1.f, cur_stream(),
              scal.data_ptr<float>());
}

void weight_pack(const at::Tensor& entries, int64_t n, int64_t max_elems) {
  CHECK_DEV(entries);
  TORCH_CHECK(entries.scalar_type() == at::kLong && entries.numel() == n * 6,
              "entries must be int64 [n, 6] (48-byte PackEntry records)");
  static_assert(sizeof(PackEntry) == 48, "PackEntry layout");
  c10::DeviceGuard guard(entries.device());
  weight_pack_launch(reinterpret_cast<const PackEntry*>(entries.data_ptr()), (int)n, max_elems,
                     cur_stream());
}

// ------------------------------------------------------------------------ codec
at::Tensor codec_absmax(const at::Tensor& x, const at::Tensor& seg) {
  CHECK_DEV(x); CHECK_F32(x);
  c10::DeviceGuard guard(x.device());
  const int nseg = (int)(seg.numel() / 2);
  at::Tensor s = at::empty({nseg}, x.options());
  codec_absmax_launch(x.data_ptr<float>(), seg.data_ptr<int64_t>(), nseg, s.data_ptr<float>(),
                      cur_stream());
  return s;
}

at::Tensor codec_encode(const at::Tensor& x, const at::Tensor& seg, const at::Tensor& scales,
                        int64_t codec) {
  CHECK_DEV(x); CHECK_F32(x);
  c10::DeviceGuard guard(x.device());
  const int nseg = (int)(seg.numel() / 2);
  at::Tensor out = at::zeros({x.numel()}, x.options().dtype(codec == 0 ? at::kHalf : at::kChar));
  codec_encode_launch(x.data_ptr<float>(), seg.data_ptr<int64_t>(), nseg, scales.data_ptr<float>(),
                      out.data_ptr(), (int)codec, x.numel(), cur_stream());
  return out;
}

void codec_decode_sum(at::Tensor out, const at::Tensor& q, const at::Tensor& scales,
                      const at::Tensor& w, const at::Tensor& seg, int64_t codec) {
  CHECK_DEV(out); CHECK_F32(out); CHECK_CONTIG(q);
  c10::DeviceGuard guard(out.device());
  const int nseg = (int)(seg.numel() / 2);
  const int world = (int)q.size(0);
  codec_decode_sum_launch(out.data_ptr<float>(), q.data_ptr(), scales.data_ptr<float>(),
                          w.data_ptr<float>(), seg.data_ptr<int64_t>(), nseg, world, (int)codec,
                          out.numel(), cur_stream());
}

// ------------------------------------------------------------------------ misc
at::Tensor bilinear_up2(const at::Tensor& x) {
  CHECK_DEV(x); CHECK_CONTIG(x); CHECK_BF16(x);
  c10::DeviceGuard guard(x.device());
  const Geo g = geo_of(x);
  at::Tensor y = at::empty(shape_with_c(g, g.C, 2), x.options());
  bilinear_up2_launch(bptr(x), bptr_mut(y), g.dims, g.N, g.D, g.H, g.W, g.C, false, cur_stream());
  return y;
}

at::Tensor bilinear_up2_bwd(const at::Tensor& dy) {
  CHECK_DEV(dy); CHECK_CONTIG(dy); CHECK_BF16(dy);
  c10::DeviceGuard guard(dy.device());
  Geo g = geo_of(dy);
  g.H /= 2; g.W /= 2; if (g.dims == 3) g.D /= 2;
  at::Tensor dx = at::empty(shape_with_c(g, g.C), dy.options());
  at::Tensor tmp = at::empty({dx.numel()}, dy.options().dtype(at::kFloat));
  bilinear_up2_bwd_launch(bptr(dy), tmp.data_ptr<float>(), bptr_mut(dx), g.dims, g.N, g.D, g.H,
                          g.W, g.C, cur_stream());
  return dx;
}

// NCHW / NCDHW tensor (fp32 or bf16; contiguous or channels_last memory) -> channel-last bf16
// [N, (D,) H, W, Cp] with channels zero-padded to a multiple of `cpad`
at::Tensor to_nhwc_bf16(const at::Tensor& x, int64_t cpad) {
  CHECK_DEV(x);
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "fp32/bf16 input");
  c10::DeviceGuard guard(x.device());
  const int N = (int)x.size(0), C = (int)x.size(1);
  const int Cp = (int)((C + cpad - 1) / cpad * cpad);
  const long long S = x.numel() / ((long long)N * C);
  // supported memory layouts: NCHW-contiguous or channel-last-contiguous
  long long sC, sS;
  if (x.is_contiguous()) { sC = S; sS = 1; }
  else {
    const auto cl = x.dim() == 4 ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::ChannelsLast3d;
    TORCH_CHECK(x.is_contiguous(cl), "input must be contiguous or channels-last");
    sC = 1; sS = C;
  }
  std::vector<int64_t> shape = {N};
  for (int i = 2; i < x.dim(); ++i) shape.push_back(x.size(i));
  shape.push_back(Cp);
  at::Tensor y = at::empty(shape, x.options().dtype(at::kBFloat16));
  to_nhwc_pad_launch(x.data_ptr(), x.scalar_type() == at::kFloat ? 0 : 1, bptr_mut(y), N, C, Cp, S,
                     x.stride(0), sC, sS, cur_stream());
  return y;
}

// ------------------------------------------------------------------------ input pipeline
std::vector<int64_t> batch_shape(int64_t B, int64_t tile, int64_t dims) {
  std::vector<int64_t> s = {B};
  for (int i = 0; i < dims; ++i) s.push_back(tile);
  return s;
}

// synthetic Vaihingen-shape batch rendered in HBM -> {x [B, (T,) T, T, cpad] bf16, y int64}
std::vector<at::Tensor> synth_tiles(const at::Tensor& idx, int64_t seed, int64_t classes,
                                    int64_t in_ch, int64_t tile, int64_t dims, int64_t grid,
                                    double k, const at::Tensor& palette, int64_t cpad) {
  CHECK_DEV(idx); CHECK_CONTIG(idx); CHECK_DEV(palette); CHECK_F32(palette); CHECK_CONTIG(palette);
  TORCH_CHECK(idx.scalar_type() == at::kLong, "idx must be int64");
  TORCH_CHECK(dims == 2 || dims == 3, "dims must be 2 or 3");
  TORCH_CHECK(in_ch >= 1 && in_ch <= 8 && cpad >= in_ch && cpad <= 8, "1 <= in_ch <= cpad <= 8");
  TORCH_CHECK(classes >= 1 && palette.numel() == classes * in_ch, "palette must be [classes][in_ch]");
  TORCH_CHECK(grid >= 1 && grid <= tile && tile >= 1, "1 <= grid <= tile");
  TORCH_CHECK((int64_t)tile * tile * (dims == 3 ? tile : 1) * 8 < (int64_t)UINT32_MAX,
              "tile too large for the 32-bit per-pixel hash counter");
  c10::DeviceGuard guard(idx.device());
  const int64_t B = idx.numel();
  std::vector<int64_t> xs = batch_shape(B, tile, dims);
  at::Tensor y = at::empty(xs, idx.options());
  xs.push_back(cpad);
  at::Tensor x = at::empty(xs, idx.options().dtype(at::kBFloat16));
  if (B > 0)
    synth_tiles_launch(idx.data_ptr<int64_t>(), (int)B, (uint32_t)(seed & 0xffffffff), (int)classes,
                       (int)in_ch, (int)tile, (int)dims, (int)grid, (float)k,
                       palette.data_ptr<float>(), (int)cpad, bptr_mut(x), y.data_ptr<int64_t>(),
                       cur_stream());
  return {x, y};
}

// HBM-resident uint8 dataset [N, (D,) H, W, Cin] + uint8 labels -> gathered bf16 / int64 batch
std::vector<at::Tensor> tile_gather(const at::Tensor& src, const at::Tensor& lab,
                                    const at::Tensor& idx, int64_t cpad) {
  CHECK_DEV(src); CHECK_CONTIG(src); CHECK_DEV(lab); CHECK_CONTIG(lab); CHECK_DEV(idx);
  CHECK_CONTIG(idx);
  TORCH_CHECK(src.scalar_type() == at::kByte && lab.scalar_type() == at::kByte, "uint8 dataset");
  TORCH_CHECK(idx.scalar_type() == at::kLong, "idx must be int64");
  TORCH_CHECK(src.dim() == lab.dim() + 1 && src.size(0) == lab.size(0), "images [N,...,C] / labels [N,...]");
  const int64_t in_ch = src.size(-1);
  TORCH_CHECK(in_ch >= 1 && in_ch <= 8 && cpad >= in_ch && cpad <= 8, "1 <= in_ch <= cpad <= 8");
  for (int64_t i = 1; i < lab.dim(); ++i) TORCH_CHECK(src.size(i) == lab.size(i), "spatial mismatch");
  c10::DeviceGuard guard(src.device());
  const int64_t B = idx.numel();
  const long long S = lab.numel() / std::max<int64_t>(1, lab.size(0));
  std::vector<int64_t> ys = {B};
  for (int64_t i = 1; i < lab.dim(); ++i) ys.push_back(lab.size(i));
  at::Tensor y = at::empty(ys, idx.options());
  std::vector<int64_t> xs = ys;
  xs.push_back(cpad);
  at::Tensor x = at::empty(xs, src.options().dtype(at::kBFloat16));
  if (B > 0)
    tile_gather_launch(src.data_ptr<uint8_t>(), lab.data_ptr<uint8_t>(), idx.data_ptr<int64_t>(),
                       (int)B, S, (int)in_ch, (int)cpad, (long long)lab.size(0), bptr_mut(x),
                       y.data_ptr<int64_t>(), cur_stream());
  return {x, y};
}

// -> the CU count grids are sized for after reserving k CUs (k < 0: query only)
int64_t set_cu_reserve(int64_t k) {
  if (k >= 0) g_cu_reserve = (int)std::min<int64_t>(k, std::max(0, phys_cus() - 8));
  return num_cus();
}

// single-GPU stand-in for a bucket all-reduce (Trainer comm_proxy): `blocks` workgroups
// stream the bucket `passes` times (read + write back, values unchanged) on the current
// stream — RCCL's footprint (a few tens of channels, each a streaming workgroup)
void comm_proxy(const at::Tensor& g, int64_t blocks, int64_t passes) {
  CHECK_DEV(g); CHECK_CONTIG(g); CHECK_F32(g);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0, "comm_proxy: 16-byte aligned buffer");
  c10::DeviceGuard guard(g.device());
  if (g.numel() == 0) return;
  comm_proxy_launch(g.data_ptr<float>(), g.numel(), (int)blocks, (int)passes, cur_stream());
}

}  // namespace

}  // namespace ddlpc

TORCH_LIBRARY(ddlpc, m) {
  m.def("set_cu_reserve(int k) -> int", &ddlpc::set_cu_reserve);
  m.def("set_knob(str name, int value) -> int", &ddlpc::set_knob);
  m.def("comm_proxy(Tensor(a!) g, int blocks, int passes) -> ()");
  m.def("conv3_fwd(Tensor x1, Tensor? x2, Tensor w, Tensor? bias, Tensor? pscale, Tensor? pshift, "
        "int cout, int co1, bool stats, Tensor? pscale2=None, Tensor? pshift2=None, Tensor? bnb_y=None, "
        "Tensor? bnb_s4=None, int groups=0) -> Tensor[]");
  m.def("conv3_wgrad(Tensor dy, Tensor x1, Tensor? x2, Tensor? pscale, Tensor? pshift, Tensor(a!)? out=None, "
        "Tensor? pscale2=None, Tensor? pshift2=None, Tensor? dy_y=None, Tensor? dy_s4=None, "
        "Tensor? dy_coefs=None, int cin_real=0, int groups=0, Tensor(b!)? dy_out=None) -> Tensor");
  m.def("conv3_bwd32(Tensor dy, Tensor y, Tensor s4, Tensor wd, Tensor(a!)? dw_out=None, int groups=0) -> Tensor[]");
  m.def("reduce_rows(Tensor partial, int R, int N) -> Tensor");
  m.def("bn_finalize(Tensor partial, float count, Tensor gamma, Tensor beta, Tensor(a!) running_mean, "
        "Tensor(b!) running_var, float momentum, float eps, bool update_running, Tensor(c!)? nbt) -> Tensor");
  m.def("bn_relu_apply(Tensor y, Tensor stats4, bool pool, bool full=True) -> Tensor[]");
  m.def("bn_running_apply(Tensor(a!) running_mean, Tensor(b!) running_var, Tensor slots, float momentum, "
        "Tensor(c!)? nbt=None) -> ()");
  m.def("bn_grad_coefs(Tensor partial, Tensor y, Tensor stats4, Tensor gamma, "
        "Tensor(a!)? dgamma_out=None, Tensor(b!)? dbeta_out=None) -> Tensor[]");
  m.def("bn_group_finalize(Tensor y, int groups, Tensor gamma, Tensor beta, float eps, "
        "Tensor(a!)? arena=None, int aoff=0) -> Tensor");
  m.def("bn_group_apply(Tensor y, Tensor stats4, int groups, bool pool) -> Tensor[]");
  m.def("bn_running_apply_all(Tensor entries, Tensor(a!) arena, int K, int maxC, float momentum) -> ()");
  m.def("bn_group_backward(Tensor? dA, Tensor? dP, Tensor y, Tensor stats4, Tensor gamma, int groups, "
        "Tensor(a!)? dgamma_out=None, Tensor(b!)? dbeta_out=None, Tensor? partial=None) -> Tensor[]");
  m.def("bn_group_finalize_rows(Tensor partial, int groups, float count, Tensor gamma, Tensor beta, "
        "float eps, Tensor(a!)? arena=None, int aoff=0) -> Tensor");
  m.def("bn_backward(Tensor? dA, Tensor? dP, Tensor y, Tensor stats4, Tensor gamma, Tensor? gscale, "
        "Tensor(a!)? dgamma_out=None, Tensor(b!)? dbeta_out=None, Tensor? partial=None) -> Tensor[]");
  m.def("convt_fwd(Tensor x, Tensor wt, Tensor? bias, int cout, Tensor? bn4=None) -> Tensor");
  m.def("convt_dgrad(Tensor dout, Tensor wd, int cin, Tensor? bny=None, Tensor? bn4=None) -> Tensor[]");
  m.def("convt_wgrad(Tensor x, Tensor dout, Tensor(a!)? dw_out=None, Tensor(b!)? db_out=None, "
        "Tensor? colsum_rows=None, Tensor? bn4=None) -> Tensor[]");
  m.def("convt_bwd_fused(Tensor x, Tensor dout, Tensor wd, Tensor(a!)? dw_out=None, "
        "Tensor(b!)? db_out=None, Tensor? colsum_rows=None, Tensor? bn4=None) -> Tensor[]");
  m.def("head_ce_fwd(Tensor a, Tensor Wh, Tensor bh, Tensor labels, int ignore_index, Tensor? bn4=None) -> Tensor");
  m.def("head_ce_bwd(Tensor a, Tensor Wh, Tensor bh, Tensor labels, Tensor out3, Tensor? gscale, "
        "int ignore_index, Tensor(a!)? dw_out=None, Tensor(b!)? db_out=None, Tensor? bn4=None, "
        "bool store_da=True) -> Tensor[]");
  m.def("head_ce_bn_bwd(Tensor a, Tensor Wh, Tensor bh, Tensor labels, Tensor out3, Tensor? gscale, "
        "int ignore_index, Tensor bn4, Tensor partial, Tensor gamma, Tensor(a!)? dgamma_out=None, "
        "Tensor(b!)? dbeta_out=None, Tensor? pscale=None, int groups=0) -> Tensor[]");
  m.def("head_ce_fwd_stats(Tensor a, Tensor Wh, Tensor bh, Tensor labels, int ignore_index, "
        "Tensor bn4, int groups=0) -> Tensor[]");
  m.def("head_wgrad_from_rows(Tensor rows, Tensor scale, int K, int C, Tensor(a!)? dw_out=None, "
        "Tensor(b!)? db_out=None) -> Tensor[]");
  m.def("meter_add(Tensor(a!) buf, Tensor loss, Tensor correct, float pixels, float count=1.) -> ()");
  m.def("head_grad_scale(Tensor out3, Tensor? gs=None) -> Tensor");
  m.def("head_logits(Tensor a, Tensor Wh, Tensor bh, Tensor? bn4=None) -> Tensor");
  m.def("adam_step(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, float b1, float b2, float eps, "
        "float wd, float step_size, float inv_sqrt_bc2) -> ()");
  m.def("adam_step_dev(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor(d!) scal, "
        "float lr, float b1, float b2, float eps, float wd) -> ()");
  m.def("weight_pack(Tensor entries, int n, int max_elems) -> ()");
  m.def("codec_absmax(Tensor x, Tensor seg) -> Tensor");
  m.def("codec_encode(Tensor x, Tensor seg, Tensor scales, int codec) -> Tensor");
  m.def("codec_decode_sum(Tensor(a!) out, Tensor q, Tensor scales, Tensor w, Tensor seg, int codec) -> ()");
  m.def("bilinear_up2(Tensor x) -> Tensor");
  m.def("bilinear_up2_bwd(Tensor dy) -> Tensor");
  m.def("to_nhwc_bf16(Tensor x, int cpad=1) -> Tensor");
  m.def("synth_tiles(Tensor idx, int seed, int classes, int in_ch, int tile, int dims, int grid, "
        "float k, Tensor palette, int cpad) -> Tensor[]");
  m.def("tile_gather(Tensor src, Tensor lab, Tensor idx, int cpad) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(ddlpc, CUDA, m) {
  m.impl("conv3_fwd", &ddlpc::conv3_fwd);
  m.impl("conv3_wgrad", &ddlpc::conv3_wgrad);
  m.impl("bn_finalize", &ddlpc::bn_finalize);
  m.impl("reduce_rows", &ddlpc::reduce_rows);
  m.impl("bn_relu_apply", &ddlpc::bn_relu_apply);
  m.impl("bn_running_apply", &ddlpc::bn_running_apply);
  m.impl("bn_grad_coefs", &ddlpc::bn_grad_coefs);
  m.impl("conv3_bwd32", &ddlpc::conv3_bwd32);
  m.impl("bn_backward", &ddlpc::bn_backward);
  m.impl("bn_group_finalize", &ddlpc::bn_group_finalize);
  m.impl("bn_group_apply", &ddlpc::bn_group_apply);
  m.impl("bn_running_apply_all", &ddlpc::bn_running_apply_all);
  m.impl("bn_group_backward", &ddlpc::bn_group_backward);
  m.impl("bn_group_finalize_rows", &ddlpc::bn_group_finalize_rows);
  m.impl("convt_fwd", &ddlpc::convt_fwd);
  m.impl("convt_dgrad", &ddlpc::convt_dgrad);
  m.impl("convt_wgrad", &ddlpc::convt_wgrad);
  m.impl("convt_bwd_fused", &ddlpc::convt_bwd_fused);
  m.impl("head_ce_fwd", &ddlpc::head_ce_fwd);
  m.impl("head_ce_bwd", &ddlpc::head_ce_bwd);
  m.impl("head_ce_bn_bwd", &ddlpc::head_ce_bn_bwd);
  m.impl("head_ce_fwd_stats", &ddlpc::head_ce_fwd_stats);
  m.impl("head_wgrad_from_rows", &ddlpc::head_wgrad_from_rows);
  m.impl("head_grad_scale", &ddlpc::head_grad_scale);
  m.impl("meter_add", &ddlpc::meter_add);
  m.impl("head_logits", &ddlpc::head_logits);
  m.impl("adam_step", &ddlpc::adam_step);
  m.impl("adam_step_dev", &ddlpc::adam_step_dev);
  m.impl("weight_pack", &ddlpc::weight_pack);
  m.impl("codec_absmax", &ddlpc::codec_absmax);
  m.impl("codec_encode", &ddlpc::codec_encode);
  m.impl("codec_decode_sum", &ddlpc::codec_decode_sum);
  m.impl("bilinear_up2", &ddlpc::bilinear_up2);
  m.impl("bilinear_up2_bwd", &ddlpc::bilinear_up2_bwd);
  m.impl("to_nhwc_bf16", &ddlpc::to_nhwc_bf16);
  m.impl("synth_tiles", &ddlpc::synth_tiles);
  m.impl("tile_gather", &ddlpc::tile_gather);
  m.impl("comm_proxy", &ddlpc::comm_proxy);
}
