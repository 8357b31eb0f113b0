// CPU kernels of the ddlpc operator namespace: TORCH_LIBRARY_IMPL(ddlpc, CPU, ...).
//
// Every operator that bindings.cpp declares (TORCH_LIBRARY(ddlpc)) and registers for the
// GPU (TORCH_LIBRARY_IMPL(ddlpc, CUDA)) gets a plain C++ / ATen reference here, with the
// same schema, the same tensor conventions and the same numerics contract: bf16
// channel-last activations [N, (D,) H, W, C], fp32 accumulation, bf16 outputs, fp64
// statistics reductions, packed bf16 weights from weight_pack.  PyTorch's dispatcher picks
// the kernel by the tensors' device, so the engine (ops/fused_unet.py) runs one code path
// on either device and a CPU-only machine trains the same model through the same ops
// (one op namespace, CPU kernel = ATen reference, device dispatch by
// PyTorch).  The GPU tests compare every op on both devices (tests/test_cpu_ops.py).
//
// Partial-row outputs ([R][2][C] statistics, [R][K*C+K] head rows) use R = 1 row (per
// group where the op is grouped): consumers sum rows, so any R is valid.
// comm_proxy has no CPU kernel: it stands in for an RCCL collective on one GPU.
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <torch/library.h>

#include <array>
#include <cmath>
#include <cstdint>
#include <vector>

namespace ddlpc_cpu {

using at::Tensor;
using c10::optional;

namespace {

bool has(const optional<Tensor>& t) { return t.has_value() && t->defined(); }
bool has_nonempty(const optional<Tensor>& t) { return has(t) && t->numel() > 0; }
Tensor f32(const Tensor& t) { return t.to(at::kFloat); }
Tensor bf(const Tensor& t) { return t.to(at::kBFloat16); }
Tensor rbf(const Tensor& t) { return t.to(at::kBFloat16).to(at::kFloat); }    // bf16 rounding
Tensor empty_f(const Tensor& like) { return at::empty({0}, like.options().dtype(at::kFloat)); }

int sdims(const Tensor& x) {
  TORCH_CHECK(x.dim() == 4 || x.dim() == 5, "expected [N,(D,)H,W,C] channel-last tensor");
  return (int)x.dim() - 2;
}
// channel-last [N, S..., C] <-> channel-first [N, C, S...]
Tensor to_cf(const Tensor& x) {
  std::vector<int64_t> p = {0, x.dim() - 1};
  for (int64_t i = 1; i < x.dim() - 1; ++i) p.push_back(i);
  return x.permute(p);
}
Tensor to_cl(const Tensor& x) {
  std::vector<int64_t> p = {0};
  for (int64_t i = 2; i < x.dim(); ++i) p.push_back(i);
  p.push_back(1);
  return x.permute(p).contiguous();
}

// rows r of stats4 [4][C] -> [C]; grouped [G][4][C] -> [G][C]
Tensor s4row(const Tensor& s4, int64_t G, int64_t C, int r) {
  if (G > 1) return s4.reshape({G, 4, C}).select(1, r);
  return s4.reshape({4, C}).select(0, r);
}

// per-channel affine of a channel-last tensor; v: [C] or, with groups, [G][C] (the batch
// holds the G groups' images one after another)
Tensor chan(const Tensor& x, const Tensor& v, int64_t G) {
  const int64_t C = x.size(-1);
  if (G > 1 && v.dim() == 2) return v.reshape({G, 1, C});
  return v.reshape({C});
}
Tensor grouped(const Tensor& x, int64_t G) {
  return G > 1 ? x.reshape({G, -1, x.size(-1)}) : x;
}
// BN + ReLU of a pre-BN tensor, rounded to bf16 as a materialised activation
Tensor bn_act(const Tensor& yf, const Tensor& scale, const Tensor& shift, int64_t G) {
  const Tensor xg = grouped(yf, G);
  return rbf(at::relu(xg * chan(yf, scale, G) + chan(yf, shift, G))).reshape(yf.sizes());
}

// packed [Cout][taps][CinW] -> fp32 OIHW / OIDHW over the first Cin input channels
Tensor unpack_w3(const Tensor& wp, int64_t cin, int dims) {
  const int64_t cout = wp.size(0);
  Tensor w = f32(wp.narrow(2, 0, cin)).permute({0, 2, 1});
  if (dims == 2) return w.reshape({cout, cin, 3, 3});
  return w.reshape({cout, cin, 3, 3, 3});
}

// (a channel-last tensor viewed channel-first IS channels_last memory: oneDNN convolves it
// in place, no layout copies)
at::MemoryFormat cl_format(int dims) {
  return dims == 2 ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::ChannelsLast3d;
}

Tensor conv_same(const Tensor& xcl, const Tensor& w, int dims) {
  const Tensor x = to_cf(xcl).contiguous(cl_format(dims));
  const Tensor y = dims == 2 ? at::conv2d(x, w, {}, 1, 1) : at::conv3d(x, w, {}, 1, 1);
  return to_cl(y);
}

Tensor wgrad_same(const Tensor& dycl, const Tensor& xcl, int dims) {
  const int64_t cout = dycl.size(-1), cin = xcl.size(-1);
  std::vector<int64_t> ws = {cout, cin, 3, 3};
  if (dims == 3) ws.push_back(3);
  const Tensor w = at::zeros(ws, xcl.options().dtype(at::kFloat));
  std::vector<int64_t> one(dims, 1), zero(dims, 0);
  auto r = at::convolution_backward(to_cf(dycl).contiguous(cl_format(dims)),
                                    to_cf(xcl).contiguous(cl_format(dims)), w.contiguous(cl_format(dims)),
                                    c10::nullopt, one, one, one, false, zero, 1,
                                    {false, true, false});
  return std::get<1>(r);
}

// (sum, sum^2) per channel -> [G][2][C] rows
Tensor stat_rows(const Tensor& yf, int64_t G) {
  const int64_t C = yf.size(-1);
  const Tensor d = yf.to(at::kDouble).reshape({G, -1, C});
  return at::stack({d.sum(1), (d * d).sum(1)}, 1).to(at::kFloat);
}

// BatchNorm-backward partial rows (sum dyh, sum dyh * xhat) of an activation gradient dA
// against the pre-BN y (ReLU mask from y * scale + shift): [G][2][C]
Tensor bnb_rows(const Tensor& dAf, const Tensor& yf, const Tensor& s4, int64_t G) {
  const int64_t C = yf.size(-1);
  const Tensor yg = grouped(yf, G), dg = grouped(dAf, G);
  const Tensor a = yg * chan(yf, s4row(s4, G, C, 2), G) + chan(yf, s4row(s4, G, C, 3), G);
  const Tensor dyh = at::where(a > 0, dg, at::zeros_like(dg)).to(at::kDouble);
  const Tensor xh = ((yg - chan(yf, s4row(s4, G, C, 0), G)) * chan(yf, s4row(s4, G, C, 1), G))
                        .to(at::kDouble);
  const Tensor d3 = dyh.reshape({G, -1, C}), x3 = xh.reshape({G, -1, C});
  return at::stack({d3.sum(1), (d3 * x3).sum(1)}, 1).to(at::kFloat);
}

// unpool a pooled gradient to the first arg-max of the bf16-rounded activation's windows
Tensor unpool(const Tensor& dPf, const Tensor& act, int dims) {
  const Tensor a = to_cf(act).contiguous();
  const Tensor g = to_cf(dPf).contiguous();
  std::vector<int64_t> k(dims, 2), zero(dims, 0), one(dims, 1);
  Tensor out;
  if (dims == 2) {
    auto r = at::max_pool2d_with_indices(a, k, k, zero, one, false);
    out = at::max_pool2d_with_indices_backward(g, a, k, k, zero, one, false, std::get<1>(r));
  } else {
    auto r = at::max_pool3d_with_indices(a, k, k, zero, one, false);
    out = at::max_pool3d_with_indices_backward(g, a, k, k, zero, one, false, std::get<1>(r));
  }
  return to_cl(out);
}

Tensor maxpool(const Tensor& act, int dims) {
  const Tensor a = to_cf(act).contiguous();
  return to_cl(dims == 2 ? at::max_pool2d(a, {2, 2}, {2, 2}) : at::max_pool3d(a, {2, 2, 2}, {2, 2, 2}));
}

// dY = k * (dyh - m1 - xhat * m2) with dyh = dt * gs where y * scale + shift > 0
struct BnBwd {
  Tensor dyh, xh;
};
BnBwd bn_terms(const Tensor& dtf, const Tensor& yf, const Tensor& s4, int64_t G, double gs) {
  const int64_t C = yf.size(-1);
  const Tensor yg = grouped(yf, G), dg = grouped(dtf, G);
  const Tensor a = yg * chan(yf, s4row(s4, G, C, 2), G) + chan(yf, s4row(s4, G, C, 3), G);
  BnBwd t;
  t.dyh = at::where(a > 0, dg * gs, at::zeros_like(dg));
  t.xh = (yg - chan(yf, s4row(s4, G, C, 0), G)) * chan(yf, s4row(s4, G, C, 1), G);
  return t;
}

// sums [G][2][C] (fp64) -> coefficients [G][3][C] = (gamma * invstd, s1 / count, s2 / count);
// dbeta / dgamma = sums over the groups, written or accumulated
Tensor bn_coefs(const Tensor& sums, const Tensor& s4, const Tensor& gamma, int64_t G, double count,
                Tensor& dgamma, Tensor& dbeta, bool into) {
  const int64_t C = gamma.numel();
  const Tensor inv = s4row(s4, G, C, 1).reshape({G, C});
  const Tensor k = gamma.reshape({1, C}) * inv;
  const Tensor m1 = (sums.select(1, 0) / count).to(at::kFloat);
  const Tensor m2 = (sums.select(1, 1) / count).to(at::kFloat);
  const Tensor db = sums.select(1, 0).sum(0).to(at::kFloat);
  const Tensor dgm = sums.select(1, 1).sum(0).to(at::kFloat);
  if (into) {
    dbeta.add_(db);
    dgamma.add_(dgm);
  } else {
    dbeta = db;
    dgamma = dgm;
  }
  return at::stack({k, m1, m2}, 1);          // [G][3][C]
}

Tensor bn_apply_coefs(const BnBwd& t, const Tensor& coefs, const Tensor& like, int64_t G) {
  const int64_t C = like.size(-1);
  const Tensor cg = coefs.reshape({G, 3, C});
  auto col = [&](int r) { return G > 1 ? cg.select(1, r).reshape({G, 1, C}) : cg.select(1, r).reshape({C}); };
  const Tensor dy = col(0) * (t.dyh - col(1) - t.xh * col(2));
  return bf(dy.reshape(like.sizes()));
}

// dst (+)= v for a caller-owned gradient buffer of v's element count (any strides)
void add_to(Tensor dst, const Tensor& v) {
  TORCH_CHECK(dst.numel() == v.numel(), "gradient out size mismatch");
  dst.add_(v.reshape(dst.sizes()));
}

double scalar_or(const optional<Tensor>& t, double d) {
  return has(t) ? t->to(at::kDouble).reshape({-1})[0].item<double>() : d;
}

// ------------------------------------------------------------------------ conv 3x3(x3)
Tensor prologue_input(const Tensor& x1, const optional<Tensor>& x2, const optional<Tensor>& ps,
                      const optional<Tensor>& sh, const optional<Tensor>& ps2,
                      const optional<Tensor>& sh2, int64_t G) {
  Tensor a = f32(x1);
  if (has(ps)) a = bn_act(a, *ps, *sh, G);
  if (has(x2)) {
    Tensor b = f32(*x2);
    if (has(ps2)) b = bn_act(b, *ps2, *sh2, 1);
    a = at::cat({a, b}, -1);
  }
  return a;
}

std::vector<Tensor> conv3_fwd(const Tensor& x1, const optional<Tensor>& x2, const Tensor& w,
                              const optional<Tensor>& bias, const optional<Tensor>& pscale,
                              const optional<Tensor>& pshift, int64_t cout, int64_t co1, bool want_stats,
                              const optional<Tensor>& pscale2, const optional<Tensor>& pshift2,
                              const optional<Tensor>& bnb_y, const optional<Tensor>& bnb_s4, int64_t groups) {
  const int dims = sdims(x1);
  const int64_t G = groups > 1 ? groups : 1;
  TORCH_CHECK(x1.size(0) % G == 0, "conv3_fwd: groups must divide the batch");
  const Tensor xin = prologue_input(x1, x2, pscale, pshift, pscale2, pshift2, G);
  TORCH_CHECK(w.dim() == 3 && w.size(0) == cout && w.size(2) >= xin.size(-1),
              "packed weight must be [Cout][taps][CinW>=Cin]");
  Tensor out = conv_same(xin, unpack_w3(w, xin.size(-1), dims), dims);
  if (has(bias)) out = out + bias->reshape({cout});
  const Tensor yb = bf(out);
  const int64_t c1 = co1 > 0 ? co1 : cout;
  const Tensor none = at::empty({0}, x1.options());
  Tensor y1 = c1 < cout ? yb.narrow(-1, 0, c1).contiguous() : yb;
  Tensor y2 = c1 < cout ? yb.narrow(-1, c1, cout - c1).contiguous() : none;
  Tensor stats = none;
  // (statistics of the fp32 outputs before the bf16 store, as the GPU epilogues reduce them)
  if (has(bnb_y)) stats = bnb_rows(out, f32(*bnb_y), *bnb_s4, G);
  else if (want_stats) stats = stat_rows(out, G);
  return {y1, y2, stats};
}

Tensor conv3_wgrad(const Tensor& dy, const Tensor& x1, const optional<Tensor>& x2,
                   const optional<Tensor>& pscale, const optional<Tensor>& pshift,
                   const optional<Tensor>& out, const optional<Tensor>& pscale2,
                   const optional<Tensor>& pshift2, const optional<Tensor>& dy_y,
                   const optional<Tensor>& dy_s4, const optional<Tensor>& dy_coefs, int64_t cin_real,
                   int64_t groups, const optional<Tensor>& dy_out) {
  (void)cin_real;                       // (the GPU's image-layer kernel choice; same result)
  const int dims = sdims(x1);
  const int64_t G = groups > 1 ? groups : 1;
  Tensor d = f32(dy);
  if (has(dy_y)) {
    // dy holds dA: BatchNorm backward applied on load with the reduced coefficients
    TORCH_CHECK(has(dy_s4) && has(dy_coefs), "conv3_wgrad: dy_s4 [4][Cout] and dy_coefs [3][Cout]");
    const BnBwd t = bn_terms(d, f32(*dy_y), *dy_s4, 1, 1.0);
    const Tensor dY = bn_apply_coefs(t, *dy_coefs, dy, 1);
    if (has(dy_out)) dy_out->copy_(dY.reshape(dy_out->sizes()));
    d = f32(dY);
  }
  TORCH_CHECK(!has(dy_out) || has(dy_y), "conv3_wgrad: dy_out needs the dY prologue");
  const Tensor xin = prologue_input(x1, x2, pscale, pshift, pscale2, pshift2, G);
  const Tensor dW = wgrad_same(d, xin, dims);
  if (has(out)) {
    TORCH_CHECK(out->numel() == dW.numel(), "dW out size mismatch");
    add_to(*out, dW);
    return empty_f(dy);
  }
  return dW;
}

std::vector<Tensor> conv3_bwd32(const Tensor& dy, const Tensor& y, const Tensor& s4, const Tensor& wd,
                                const optional<Tensor>& dw_out, int64_t groups) {
  const int64_t G = groups > 1 ? groups : 1;
  const int64_t C = y.size(-1);
  const Tensor yf = f32(y);
  const Tensor dAf = conv_same(f32(dy), unpack_w3(wd, dy.size(-1), 2), 2);
  const Tensor dA = bf(dAf);
  const Tensor part = bnb_rows(dAf, yf, s4, G);
  const Tensor x = bn_act(yf, s4row(s4, G, C, 2), s4row(s4, G, C, 3), G);
  const Tensor dW = wgrad_same(f32(dy), x, 2);
  if (has(dw_out)) {
    add_to(*dw_out, dW);
    return {dA, part, empty_f(dy)};
  }
  return {dA, part, dW};
}

Tensor reduce_rows(const Tensor& partial, int64_t R, int64_t N) {
  return partial.reshape({R, N}).to(at::kDouble).sum(0);
}

// ------------------------------------------------------------------------ BatchNorm
float mom_update(float running, float x, float m) { return m * x + (1.f - m) * running; }

// stats4 [G][4][C] from fp64 sums [G][2][C]; arena rows (mean | unbiased var) if given
Tensor stats4_from_sums(const Tensor& sums, double count, const Tensor& gamma, const Tensor& beta,
                        double eps, int64_t G, float* arena, int64_t astride) {
  const int64_t C = gamma.numel();
  Tensor st = at::empty({G, 4, C}, gamma.options());
  const auto S = sums.contiguous();
  const double* s = S.data_ptr<double>();
  const Tensor gc = gamma.contiguous(), bc = beta.contiguous();
  const float* g = gc.data_ptr<float>();
  const float* b = bc.data_ptr<float>();
  float* o = st.data_ptr<float>();
  for (int64_t k = 0; k < G; ++k)
    for (int64_t c = 0; c < C; ++c) {
      const double mean = s[(k * 2) * C + c] / count;
      double var = s[(k * 2 + 1) * C + c] / count - mean * mean;
      if (var < 0) var = 0;
      const float inv = (float)(1.0 / std::sqrt(var + eps));
      const float sc = g[c] * inv;
      float* ok = o + k * 4 * C;
      ok[c] = (float)mean;
      ok[C + c] = inv;
      ok[2 * C + c] = sc;
      ok[3 * C + c] = b[c] - (float)mean * sc;
      if (arena != nullptr) {
        arena[k * astride + c] = (float)mean;
        arena[k * astride + C + c] = (float)(count > 1 ? var * count / (count - 1) : var);
      }
    }
  return st;
}

Tensor bn_finalize(const Tensor& partial, double count, const Tensor& gamma, const Tensor& beta,
                   Tensor running_mean, Tensor running_var, double momentum, double eps,
                   bool update_running, const optional<Tensor>& nbt) {
  const int64_t C = gamma.numel();
  const Tensor sums = partial.reshape({-1, 2, C}).to(at::kDouble).sum(0, true);
  Tensor arena;
  float* ap = nullptr;
  if (update_running) {
    arena = at::empty({2 * C}, gamma.options());
    ap = arena.data_ptr<float>();
  }
  const Tensor st = stats4_from_sums(sums, count, gamma, beta, eps, 1, ap, 0).reshape({4, C});
  if (update_running) {
    float* rm = running_mean.data_ptr<float>();
    float* rv = running_var.data_ptr<float>();
    for (int64_t c = 0; c < C; ++c) {
      rm[c] = mom_update(rm[c], ap[c], (float)momentum);
      rv[c] = mom_update(rv[c], ap[C + c], (float)momentum);
    }
    if (has(nbt)) nbt->add_(1);
  }
  return st;
}

void bn_running_apply(Tensor running_mean, Tensor running_var, const Tensor& slots, double momentum,
                      const optional<Tensor>& nbt) {
  const int64_t C = running_mean.numel(), K = slots.size(0);
  TORCH_CHECK(slots.dim() == 2 && slots.size(1) == 2 * C && slots.stride(1) == 1, "slots [K][2C]");
  float* rm = running_mean.data_ptr<float>();
  float* rv = running_var.data_ptr<float>();
  const float* s = slots.data_ptr<float>();
  for (int64_t c = 0; c < C; ++c)
    for (int64_t k = 0; k < K; ++k) {
      rm[c] = mom_update(rm[c], s[k * slots.stride(0) + c], (float)momentum);
      rv[c] = mom_update(rv[c], s[k * slots.stride(0) + C + c], (float)momentum);
    }
  if (has(nbt) && K > 0) nbt->add_(K);
}

void bn_running_apply_all(const Tensor& entries, const Tensor& arena, int64_t K, int64_t maxC, double momentum) {
  (void)maxC;
  TORCH_CHECK(entries.scalar_type() == at::kLong && entries.dim() == 2 && entries.size(1) == 4,
              "entries [L][4] int64");
  const Tensor e = entries.contiguous();
  const int64_t* ep = e.data_ptr<int64_t>();
  const float* a = arena.data_ptr<float>();
  const int64_t stride = arena.stride(0);
  for (int64_t l = 0; l < e.size(0); ++l) {
    float* rm = reinterpret_cast<float*>(ep[4 * l]);
    float* rv = reinterpret_cast<float*>(ep[4 * l + 1]);
    int64_t* nb = reinterpret_cast<int64_t*>(ep[4 * l + 2]);
    const int64_t C = ep[4 * l + 3] & 0xffffffff;
    const int64_t off = (int64_t)((uint64_t)ep[4 * l + 3] >> 32);
    if (nb != nullptr) nb[0] += K;
    for (int64_t c = 0; c < C; ++c)
      for (int64_t k = 0; k < K; ++k) {
        rm[c] = mom_update(rm[c], a[k * stride + off + c], (float)momentum);
        rv[c] = mom_update(rv[c], a[k * stride + off + C + c], (float)momentum);
      }
  }
}

std::vector<Tensor> relu_apply_groups(const Tensor& y, const Tensor& stats4, int64_t G, bool pool, bool full) {
  const int64_t C = y.size(-1);
  const Tensor a = bn_act(f32(y), s4row(stats4, G, C, 2), s4row(stats4, G, C, 3), G);
  const Tensor none = at::empty({0}, y.options());
  return {full ? bf(a) : none, pool ? bf(maxpool(a, sdims(y))) : none};
}

std::vector<Tensor> bn_relu_apply(const Tensor& y, const Tensor& stats4, bool pool, bool full) {
  TORCH_CHECK(full || pool, "bn_relu_apply: full=False only with pool (deferred skip)");
  return relu_apply_groups(y, stats4, 1, pool, full);
}

// dA (+ unpool(dP)) through ReLU and BN, per group; partial rows replace the reduction
std::vector<Tensor> bn_backward_groups(const optional<Tensor>& dA, const optional<Tensor>& dP, const Tensor& y,
                                       const Tensor& stats4, const Tensor& gamma, int64_t G, double gs,
                                       const optional<Tensor>& dgamma_out, const optional<Tensor>& dbeta_out,
                                       const optional<Tensor>& partial) {
  const bool hasA = has(dA), hasP = has(dP);
  TORCH_CHECK(hasA || hasP, "bn_backward needs dA or dP");
  const int64_t C = y.size(-1);
  const Tensor yf = f32(y);
  Tensor dt = hasA ? f32(*dA).reshape(y.sizes()) : at::zeros_like(yf);
  if (hasP) {
    const Tensor act = bn_act(yf, s4row(stats4, G, C, 2), s4row(stats4, G, C, 3), G);
    dt = dt + unpool(f32(*dP), act, sdims(y));
  }
  const BnBwd t = bn_terms(dt, yf, stats4, G, gs);
  Tensor sums;
  if (has_nonempty(partial)) {
    sums = partial->reshape({G, -1, 2, C}).to(at::kDouble).sum(1);
  } else {
    const Tensor d3 = t.dyh.to(at::kDouble).reshape({G, -1, C});
    const Tensor x3 = t.xh.to(at::kDouble).reshape({G, -1, C});
    sums = at::stack({d3.sum(1), (d3 * x3).sum(1)}, 1);
  }
  const bool into = has(dgamma_out);
  Tensor dgamma = into ? *dgamma_out : Tensor(), dbeta = into ? *dbeta_out : Tensor();
  const double count = (double)(y.numel() / C / G);
  const Tensor coefs = bn_coefs(sums, stats4, gamma, G, count, dgamma, dbeta, into);
  return {bn_apply_coefs(t, coefs, y, G), dgamma, dbeta};
}

std::vector<Tensor> bn_backward(const optional<Tensor>& dA, const optional<Tensor>& dP, const Tensor& y,
                                const Tensor& stats4, const Tensor& gamma, const optional<Tensor>& gscale,
                                const optional<Tensor>& dgamma_out, const optional<Tensor>& dbeta_out,
                                const optional<Tensor>& partial_in) {
  if (has_nonempty(partial_in))
    TORCH_CHECK(!has(dP) && !has(gscale), "precomputed BN partials: no pool / grad scale");
  return bn_backward_groups(dA, dP, y, stats4, gamma, 1, scalar_or(gscale, 1.0), dgamma_out, dbeta_out,
                            partial_in);
}

std::vector<Tensor> bn_grad_coefs(const Tensor& partial, const Tensor& y, const Tensor& stats4, const Tensor& gamma,
                                  const optional<Tensor>& dgamma_out, const optional<Tensor>& dbeta_out) {
  const int64_t C = y.size(-1);
  const Tensor sums = partial.reshape({1, -1, 2, C}).to(at::kDouble).sum(1);
  const bool into = has(dgamma_out);
  Tensor dgamma = into ? *dgamma_out : Tensor(), dbeta = into ? *dbeta_out : Tensor();
  const Tensor coefs = bn_coefs(sums, stats4, gamma, 1, (double)(y.numel() / C), dgamma, dbeta, into);
  return {coefs.reshape({3, C}), dgamma, dbeta};
}

std::pair<float*, int64_t> arena_ptr(const optional<Tensor>& arena, int64_t aoff) {
  if (!has(arena)) return {nullptr, 0};
  TORCH_CHECK(arena->dim() == 2 && arena->stride(1) == 1, "arena [rows][cols]");
  return {arena->data_ptr<float>() + aoff, arena->stride(0)};
}

Tensor bn_group_finalize(const Tensor& y, int64_t groups, const Tensor& gamma, const Tensor& beta, double eps,
                         const optional<Tensor>& arena, int64_t aoff) {
  const int64_t C = y.size(-1);
  const Tensor d = f32(y).to(at::kDouble).reshape({groups, -1, C});
  const Tensor sums = at::stack({d.sum(1), (d * d).sum(1)}, 1);
  auto ap = arena_ptr(arena, aoff);
  return stats4_from_sums(sums, (double)d.size(1), gamma, beta, eps, groups, ap.first, ap.second);
}

Tensor bn_group_finalize_rows(const Tensor& partial, int64_t groups, double count, const Tensor& gamma,
                              const Tensor& beta, double eps, const optional<Tensor>& arena, int64_t aoff) {
  const int64_t C = gamma.numel();
  const Tensor sums = partial.reshape({groups, -1, 2, C}).to(at::kDouble).sum(1);
  auto ap = arena_ptr(arena, aoff);
  return stats4_from_sums(sums, count, gamma, beta, eps, groups, ap.first, ap.second);
}

std::vector<Tensor> bn_group_apply(const Tensor& y, const Tensor& stats4, int64_t groups, bool pool) {
  return relu_apply_groups(y, stats4, groups, pool, true);
}

std::vector<Tensor> bn_group_backward(const optional<Tensor>& dA, const optional<Tensor>& dP, const Tensor& y,
                                      const Tensor& stats4, const Tensor& gamma, int64_t groups,
                                      const optional<Tensor>& dgamma_out, const optional<Tensor>& dbeta_out,
                                      const optional<Tensor>& partial) {
  return bn_backward_groups(dA, dP, y, stats4, gamma, groups, 1.0, dgamma_out, dbeta_out, partial);
}

// ------------------------------------------------------------------------ transposed conv
// [M][S*cout] GEMM columns (sub-position major) <-> the 2x-up-sampled channel-last tensor
Tensor shuffle_up(const Tensor& cols, const Tensor& x, int64_t cout) {
  const int dims = sdims(x);
  const int64_t N = x.size(0);
  if (dims == 2) {
    const int64_t H = x.size(1), W = x.size(2);
    return cols.reshape({N, H, W, 2, 2, cout}).permute({0, 1, 3, 2, 4, 5}).reshape({N, 2 * H, 2 * W, cout});
  }
  const int64_t D = x.size(1), H = x.size(2), W = x.size(3);
  return cols.reshape({N, D, H, W, 2, 2, 2, cout}).permute({0, 1, 4, 2, 5, 3, 6, 7})
      .reshape({N, 2 * D, 2 * H, 2 * W, cout});
}
Tensor shuffle_down(const Tensor& dout) {          // -> [M][S*cout]
  const int dims = sdims(dout);
  const int64_t N = dout.size(0), co = dout.size(-1);
  if (dims == 2) {
    const int64_t H = dout.size(1) / 2, W = dout.size(2) / 2;
    return dout.reshape({N, H, 2, W, 2, co}).permute({0, 1, 3, 2, 4, 5}).reshape({N * H * W, 4 * co});
  }
  const int64_t D = dout.size(1) / 2, H = dout.size(2) / 2, W = dout.size(3) / 2;
  return dout.reshape({N, D, 2, H, 2, W, 2, co}).permute({0, 1, 3, 5, 2, 4, 6, 7})
      .reshape({N * D * H * W, 8 * co});
}
Tensor convt_input(const Tensor& x, const optional<Tensor>& bn4) {
  const int64_t C = x.size(-1);
  if (!has(bn4)) return f32(x);
  TORCH_CHECK(bn4->numel() == 4 * C, "bn4 must be [4][C] (mean, invstd, scale, shift)");
  return bn_act(f32(x), s4row(*bn4, 1, C, 2), s4row(*bn4, 1, C, 3), 1);
}

Tensor convt_fwd(const Tensor& x, const Tensor& wt, const optional<Tensor>& bias, int64_t cout,
                 const optional<Tensor>& bn4) {
  const int64_t C = x.size(-1);
  const Tensor xin = convt_input(x, bn4).reshape({-1, C});
  const Tensor cols = at::matmul(xin, f32(wt).reshape({-1, C}).t());
  Tensor out = shuffle_up(cols, x, cout);
  if (has(bias)) out = out + bias->reshape({cout});
  return bf(out);
}

std::vector<Tensor> convt_dgrad(const Tensor& dout, const Tensor& wd, int64_t cin, const optional<Tensor>& bny,
                                const optional<Tensor>& bn4) {
  const Tensor cols = shuffle_down(f32(dout));
  std::vector<int64_t> xs = dout.sizes().vec();
  for (size_t i = 1; i + 1 < xs.size(); ++i) xs[i] /= 2;
  xs.back() = cin;
  const Tensor dxf = at::matmul(cols, f32(wd).reshape({cin, -1}).t()).reshape(xs);
  const Tensor dx = bf(dxf);
  if (!has(bn4)) return {dx, empty_f(dout)};
  TORCH_CHECK(has(bny), "convt_dgrad: bny must be the deferred pre-BN input");
  return {dx, bnb_rows(dxf, f32(*bny), *bn4, 1)};
}

Tensor convt_bias(const Tensor& dout, const optional<Tensor>& colsum_rows) {
  const int64_t co = dout.size(-1);
  if (has_nonempty(colsum_rows))
    return colsum_rows->select(1, 0).narrow(1, 0, co).to(at::kDouble).sum(0).to(at::kFloat);
  return f32(dout).reshape({-1, co}).to(at::kDouble).sum(0).to(at::kFloat);
}

std::vector<Tensor> convt_wgrad(const Tensor& x, const Tensor& dout, const optional<Tensor>& dw_out,
                                const optional<Tensor>& db_out, const optional<Tensor>& colsum_rows,
                                const optional<Tensor>& bn4) {
  const int dims = sdims(x);
  const int64_t C = x.size(-1), co = dout.size(-1), S = dims == 2 ? 4 : 8;
  const Tensor xin = convt_input(x, bn4).reshape({-1, C});
  const Tensor cols = shuffle_down(f32(dout));                     // [M][S*co]
  std::vector<int64_t> ws = {C, co, 2, 2};
  if (dims == 3) ws.push_back(2);
  const Tensor dW = at::matmul(xin.t(), cols).reshape({C, S, co}).permute({0, 2, 1}).contiguous().reshape(ws);
  const Tensor db = convt_bias(dout, colsum_rows);
  if (has(dw_out)) {
    add_to(*dw_out, dW);
    add_to(*db_out, db);
    return {empty_f(x), empty_f(x)};
  }
  return {dW, db};
}

std::vector<Tensor> convt_bwd_fused(const Tensor& x, const Tensor& dout, const Tensor& wd,
                                    const optional<Tensor>& dw_out, const optional<Tensor>& db_out,
                                    const optional<Tensor>& colsum_rows, const optional<Tensor>& bn4) {
  auto r = convt_dgrad(dout, wd, x.size(-1), has(bn4) ? optional<Tensor>(x) : c10::nullopt, bn4);
  auto w = convt_wgrad(x, dout, dw_out, db_out, colsum_rows, bn4);
  return {r[0], r[1], w[0], w[1]};
}

// ------------------------------------------------------------------------ head + CE
// the head's input activation: bf16 a, or relu(bn(y)) rounded to bf16 (deferred BN,
// per group with [G][4][C] statistics)
Tensor head_act(const Tensor& a, const optional<Tensor>& bn4, int64_t G) {
  const int64_t C = a.size(-1);
  if (!has(bn4)) return f32(a).reshape({-1, C});
  return bn_act(f32(a), s4row(*bn4, G, C, 2), s4row(*bn4, G, C, 3), G).reshape({-1, C});
}

struct HeadFwd {
  Tensor A, logits, valid, lab, out3;
};
HeadFwd head_forward(const Tensor& a, const Tensor& Wh, const Tensor& bh, const Tensor& labels,
                     int64_t ignore_index, const optional<Tensor>& bn4, int64_t G) {
  const int64_t K = Wh.size(0);
  HeadFwd h;
  h.A = head_act(a, bn4, G);
  h.logits = at::matmul(h.A, f32(Wh).reshape({K, -1}).t()) + f32(bh).reshape({K});
  const Tensor lab = labels.reshape({-1});
  h.valid = lab != ignore_index;
  h.lab = at::where(h.valid, lab, at::zeros_like(lab));
  const Tensor lse = at::logsumexp(h.logits, 1);
  const Tensor picked = h.logits.gather(1, h.lab.unsqueeze(1)).squeeze(1);
  const Tensor ce = at::where(h.valid, lse - picked, at::zeros_like(lse)).to(at::kDouble);
  const double count = h.valid.sum().item<double>();
  const double correct = (h.logits.argmax(1) == lab).sum().item<double>();
  const double loss = count > 0 ? ce.sum().item<double>() / count : 0.0;
  h.out3 = at::tensor({(float)loss, (float)correct, (float)count}, a.options().dtype(at::kFloat));
  return h;
}
// dlogits = (softmax - onehot) * scale on valid pixels
Tensor head_dlogits(const HeadFwd& h, double scale) {
  Tensor p = at::softmax(h.logits, 1);
  p = p - at::one_hot(h.lab, h.logits.size(1)).to(at::kFloat);
  return at::where(h.valid.unsqueeze(1), p * scale, at::zeros_like(p));
}
double head_scale(const Tensor& out3, const optional<Tensor>& gs) {
  const double cnt = out3[2].item<double>();
  return scalar_or(gs, 1.0) / (cnt > 0 ? cnt : 1.0);
}
void add_into(const optional<Tensor>& dst, const Tensor& v) { add_to(*dst, v); }

Tensor head_ce_fwd(const Tensor& a, const Tensor& Wh, const Tensor& bh, const Tensor& labels,
                   int64_t ignore_index, const optional<Tensor>& bn4) {
  return head_forward(a, Wh, bh, labels, ignore_index, bn4, 1).out3;
}

std::vector<Tensor> head_ce_bwd(const Tensor& a, const Tensor& Wh, const Tensor& bh, const Tensor& labels,
                                const Tensor& out3, const optional<Tensor>& gscale, int64_t ignore_index,
                                const optional<Tensor>& dw_out, const optional<Tensor>& db_out,
                                const optional<Tensor>& bn4, bool store_da) {
  TORCH_CHECK(store_da || has(bn4), "head_ce_bwd: store_da=False needs the deferred BN (bn4)");
  const int64_t K = Wh.size(0), C = a.size(-1);
  const HeadFwd h = head_forward(a, Wh, bh, labels, ignore_index, bn4, 1);
  const Tensor dl = head_dlogits(h, head_scale(out3, gscale));
  const Tensor dAf = at::matmul(dl, f32(Wh).reshape({K, C}));
  const Tensor dA = store_da ? bf(dAf.reshape(a.sizes())) : at::empty({0}, a.options());
  const Tensor dW = at::matmul(dl.t(), h.A), db = dl.sum(0);
  const Tensor bnpart = has(bn4) ? bnb_rows(rbf(dAf).reshape(a.sizes()), f32(a), *bn4, 1) : empty_f(a);
  if (has(dw_out)) {
    add_into(dw_out, dW);
    add_into(db_out, db);
    return {dA, empty_f(a), empty_f(a), bnpart};
  }
  return {dA, dW, db, bnpart};
}

std::vector<Tensor> head_ce_bn_bwd(const Tensor& a, const Tensor& Wh, const Tensor& bh, const Tensor& labels,
                                   const Tensor& out3, const optional<Tensor>& gscale, int64_t ignore_index,
                                   const Tensor& bn4, const Tensor& partial, const Tensor& gamma,
                                   const optional<Tensor>& dgamma_out, const optional<Tensor>& dbeta_out,
                                   const optional<Tensor>& pscale, int64_t groups) {
  const int64_t G = groups > 1 ? groups : 1;
  const int64_t K = Wh.size(0), C = a.size(-1);
  const HeadFwd h = head_forward(a, Wh, bh, labels, ignore_index, bn4, G);
  const Tensor dl = head_dlogits(h, head_scale(out3, gscale));
  const Tensor dAf = rbf(at::matmul(dl, f32(Wh).reshape({K, C}))).reshape(a.sizes());
  const BnBwd t = bn_terms(dAf, f32(a), bn4, G, 1.0);
  const Tensor sums = partial.reshape({G, -1, 2, C}).to(at::kDouble).sum(1) * scalar_or(pscale, 1.0);
  const bool into = has(dgamma_out);
  Tensor dgamma = into ? *dgamma_out : Tensor(), dbeta = into ? *dbeta_out : Tensor();
  const Tensor coefs = bn_coefs(sums, bn4, gamma, G, (double)(a.numel() / C / G), dgamma, dbeta, into);
  return {bn_apply_coefs(t, coefs, a, G), dgamma, dbeta};
}

std::vector<Tensor> head_ce_fwd_stats(const Tensor& a, const Tensor& Wh, const Tensor& bh, const Tensor& labels,
                                      int64_t ignore_index, const Tensor& bn4, int64_t groups) {
  const int64_t G = groups > 1 ? groups : 1;
  const int64_t K = Wh.size(0), C = a.size(-1);
  const HeadFwd h = head_forward(a, Wh, bh, labels, ignore_index, bn4, G);
  const Tensor dl = head_dlogits(h, 1.0);                   // unit gradient scale
  const Tensor dAf = rbf(at::matmul(dl, f32(Wh).reshape({K, C}))).reshape(a.sizes());
  const Tensor wrows = at::cat({at::matmul(dl.t(), h.A).reshape({-1}), dl.sum(0)}).reshape({1, K * C + K});
  return {h.out3, wrows, bnb_rows(dAf, f32(a), bn4, G)};
}

std::vector<Tensor> head_wgrad_from_rows(const Tensor& rows, const Tensor& scale, int64_t K, int64_t C,
                                         const optional<Tensor>& dw_out, const optional<Tensor>& db_out) {
  const Tensor s = (rows.to(at::kDouble).sum(0) * scale.to(at::kDouble).reshape({-1})[0]).to(at::kFloat);
  if (has(dw_out)) {
    add_into(dw_out, s.narrow(0, 0, K * C));
    add_into(db_out, s.narrow(0, K * C, K));
    return {empty_f(rows), empty_f(rows)};
  }
  return {s.narrow(0, 0, K * C).reshape({K, C}), s.narrow(0, K * C, K)};
}

Tensor head_grad_scale(const Tensor& out3, const optional<Tensor>& gs) {
  return at::tensor({(float)head_scale(out3, gs)}, out3.options());
}

void meter_add(Tensor& buf, const Tensor& loss, const Tensor& correct, double pixels, double count) {
  TORCH_CHECK(buf.scalar_type() == at::kDouble && buf.numel() == 4, "meter buffer must be 4 doubles");
  double* b = buf.data_ptr<double>();
  b[0] += loss.to(at::kDouble).item<double>() * count;
  b[1] += correct.to(at::kDouble).item<double>();
  b[2] += pixels;
  b[3] += count;
}

Tensor head_logits(const Tensor& a, const Tensor& Wh, const Tensor& bh, const optional<Tensor>& bn4) {
  const int64_t K = Wh.size(0);
  const Tensor A = head_act(a, bn4, 1);
  const Tensor l = at::matmul(A, f32(Wh).reshape({K, -1}).t()) + f32(bh).reshape({K});
  std::vector<int64_t> s = a.sizes().vec();
  s.back() = K;
  return to_cf(l.reshape(s)).contiguous();
}

// ------------------------------------------------------------------------ optimizer / pack
void adam_math(Tensor p, const Tensor& g, Tensor m, Tensor v, double b1, double b2, double eps, double wd,
               float step_size, float inv_sqrt_bc2) {
  float* P = p.data_ptr<float>();
  const Tensor gc = g.contiguous();
  const float* G = gc.data_ptr<float>();
  float* M = m.data_ptr<float>();
  float* V = v.data_ptr<float>();
  const float fb1 = (float)b1, fb2 = (float)b2, feps = (float)eps, fwd = (float)wd;
  const int64_t n = p.numel();
  at::parallel_for(0, n, 16384, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) {
      const float gr = fwd != 0.f ? G[i] + fwd * P[i] : G[i];
      M[i] = M[i] + (1.f - fb1) * (gr - M[i]);
      V[i] = fb2 * V[i] + (1.f - fb2) * gr * gr;
      P[i] = P[i] - step_size * M[i] / (std::sqrt(V[i]) * inv_sqrt_bc2 + feps);
    }
  });
}

void adam_step(Tensor p, const Tensor& g, Tensor m, Tensor v, double b1, double b2, double eps, double wd,
               double step_size, double inv_sqrt_bc2) {
  TORCH_CHECK(p.is_contiguous() && m.is_contiguous() && v.is_contiguous(), "adam: contiguous buffers");
  adam_math(p, g, m, v, b1, b2, eps, wd, (float)step_size, (float)inv_sqrt_bc2);
}

void adam_step_dev(Tensor p, const Tensor& g, Tensor m, Tensor v, Tensor scal, double lr, double b1, double b2,
                   double eps, double wd) {
  float* s = scal.data_ptr<float>();
  const double t = (double)s[0] + 1.0;
  s[0] = (float)t;
  s[1] = (float)(lr / (1.0 - std::pow(b1, t)));
  s[2] = (float)(1.0 / std::sqrt(1.0 - std::pow(b2, t)));
  adam_math(p, g, m, v, b1, b2, eps, wd, s[1], s[2]);
}

// fp32 OIHW / IOHW parameters -> bf16 kernel layouts (see csrc/misc.hip weight_pack_kernel):
// entries [n][6] = (src*, fwd*, dgrad* | 0, kind | Cout << 32, Cin | taps << 32, CinW | CoutW << 32)
void weight_pack(const Tensor& entries, int64_t n, int64_t max_elems) {
  (void)max_elems;
  TORCH_CHECK(entries.scalar_type() == at::kLong && entries.numel() == n * 6, "entries must be int64 [n, 6]");
  const Tensor e = entries.contiguous();
  const int64_t* ep = e.data_ptr<int64_t>();
  for (int64_t i = 0; i < n; ++i) {
    const int64_t* r = ep + 6 * i;
    const float* src = reinterpret_cast<const float*>(r[0]);
    auto* fwd = reinterpret_cast<c10::BFloat16*>(r[1]);
    auto* dgr = reinterpret_cast<c10::BFloat16*>(r[2]);
    const int kind = (int)(r[3] & 0xffffffff);
    const int64_t Cout = (int64_t)((uint64_t)r[3] >> 32), Cin = r[4] & 0xffffffff;
    const int64_t T = (int64_t)((uint64_t)r[4] >> 32), CinW = r[5] & 0xffffffff;
    const int64_t CoutW = (int64_t)((uint64_t)r[5] >> 32);
    if (kind == 0) {                  // OIHW [co][ci][tap]
      for (int64_t co = 0; co < Cout; ++co)
        for (int64_t ci = 0; ci < Cin; ++ci)
          for (int64_t t = 0; t < T; ++t) {
            const float v = src[(co * Cin + ci) * T + t];
            fwd[(co * T + t) * CinW + ci] = c10::BFloat16(v);
            if (dgr != nullptr) dgr[(ci * T + (T - 1 - t)) * CoutW + co] = c10::BFloat16(v);
          }
    } else {                          // IOHW [ci][co][sub]
      for (int64_t ci = 0; ci < Cin; ++ci)
        for (int64_t co = 0; co < Cout; ++co)
          for (int64_t s = 0; s < T; ++s) {
            const float v = src[(ci * Cout + co) * T + s];
            fwd[(s * Cout + co) * Cin + ci] = c10::BFloat16(v);
            if (dgr != nullptr) dgr[(ci * T + s) * Cout + co] = c10::BFloat16(v);
          }
    }
  }
}

// ------------------------------------------------------------------------ codec
std::vector<std::pair<int64_t, int64_t>> segments(const Tensor& seg) {
  const Tensor s = seg.to(at::kLong).contiguous();
  const int64_t* p = s.data_ptr<int64_t>();
  std::vector<std::pair<int64_t, int64_t>> out;
  for (int64_t i = 0; i + 1 < s.numel(); i += 2) out.emplace_back(p[i], p[i + 1]);
  return out;
}

Tensor codec_absmax(const Tensor& x, const Tensor& seg) {
  const auto segs = segments(seg);
  Tensor s = at::zeros({(int64_t)segs.size()}, x.options());
  for (size_t k = 0; k < segs.size(); ++k)
    if (segs[k].second > segs[k].first)
      s[k] = x.narrow(0, segs[k].first, segs[k].second - segs[k].first).abs().max();
  return s;
}

Tensor codec_encode(const Tensor& x, const Tensor& seg, const Tensor& scales, int64_t codec) {
  const auto segs = segments(seg);
  const float L = codec == 0 ? 100.f : 10.f;
  Tensor out = at::zeros({x.numel()}, x.options().dtype(codec == 0 ? at::kHalf : at::kChar));
  const Tensor sc = scales.contiguous();
  for (size_t k = 0; k < segs.size(); ++k) {
    const int64_t a = segs[k].first, len = segs[k].second - segs[k].first;
    const float s = sc.data_ptr<float>()[k];
    if (len <= 0 || !(s > 0.f)) continue;
    const Tensor q = at::round(x.narrow(0, a, len) / s * L);      // round half to even
    out.narrow(0, a, len).copy_(q);
  }
  return out;
}

void codec_decode_sum(Tensor out, const Tensor& q, const Tensor& scales, const Tensor& w, const Tensor& seg,
                      int64_t codec) {
  const auto segs = segments(seg);
  const float L = codec == 0 ? 100.f : 10.f;
  const int64_t world = q.size(0), n = out.numel();
  const Tensor sc = scales.reshape({world, -1});
  const Tensor qf = f32(q.reshape({world, n}));
  for (size_t k = 0; k < segs.size(); ++k) {
    const int64_t a = segs[k].first, len = segs[k].second - segs[k].first;
    if (len <= 0) continue;
    Tensor acc = at::zeros({len}, out.options());
    for (int64_t r = 0; r < world; ++r)
      acc = acc + w[r] * (qf[r].narrow(0, a, len) / L * sc[r][(int64_t)k]);
    out.narrow(0, a, len).copy_(acc);
  }
}

// ------------------------------------------------------------------------ misc
Tensor bilinear_up2(const Tensor& x) {
  const Tensor xc = to_cf(f32(x)).contiguous();
  Tensor y;
  if (x.dim() == 4)
    y = at::upsample_bilinear2d(xc, {2 * x.size(1), 2 * x.size(2)}, true);
  else
    y = at::upsample_trilinear3d(xc, {2 * x.size(1), 2 * x.size(2), 2 * x.size(3)}, true);
  return bf(to_cl(y));
}

Tensor bilinear_up2_bwd(const Tensor& dy) {
  const Tensor g = to_cf(f32(dy)).contiguous();
  Tensor dx;
  if (dy.dim() == 4) {
    const int64_t H = dy.size(1) / 2, W = dy.size(2) / 2;
    dx = at::upsample_bilinear2d_backward(g, {2 * H, 2 * W}, {dy.size(0), dy.size(3), H, W}, true);
  } else {
    const int64_t D = dy.size(1) / 2, H = dy.size(2) / 2, W = dy.size(3) / 2;
    dx = at::upsample_trilinear3d_backward(g, {2 * D, 2 * H, 2 * W}, {dy.size(0), dy.size(4), D, H, W}, true);
  }
  return bf(to_cl(dx));
}

Tensor to_nhwc_bf16(const Tensor& x, int64_t cpad) {
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "fp32/bf16 input");
  const int64_t C = x.size(1), Cp = (C + cpad - 1) / cpad * cpad;
  Tensor y = to_cl(x.to(at::kBFloat16));
  if (Cp > C) y = at::constant_pad_nd(y, {0, Cp - C}, 0);
  return y.contiguous();
}

uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
float u24(uint32_t h) { return (float)(h >> 8) * (1.0f / 16777216.0f); }

// the synthetic Vaihingen-shape batch (csrc/data.hip synth_tiles_kernel), bit for bit: every
// float operation rounds on its own (no contraction on this path)
std::vector<Tensor> synth_tiles(const Tensor& idx, int64_t seed, int64_t classes, int64_t in_ch, int64_t tile,
                                int64_t dims, int64_t grid, double k, const Tensor& palette, int64_t cpad) {
  TORCH_CHECK(dims == 2 || dims == 3, "dims must be 2 or 3");
  TORCH_CHECK(in_ch >= 1 && in_ch <= 8 && cpad >= in_ch && cpad <= 8, "1 <= in_ch <= cpad <= 8");
  TORCH_CHECK(classes >= 1 && palette.numel() == classes * in_ch, "palette must be [classes][in_ch]");
  const Tensor ix = idx.to(at::kLong).contiguous();
  const int64_t B = ix.numel();
  const int64_t S = dims == 3 ? tile * tile * tile : tile * tile;
  std::vector<int64_t> ys = {B};
  for (int i = 0; i < dims; ++i) ys.push_back(tile);
  Tensor y = at::empty(ys, idx.options().dtype(at::kLong));
  std::vector<int64_t> xs = ys;
  xs.push_back(cpad);
  Tensor x = at::empty(xs, idx.options().dtype(at::kBFloat16));
  const Tensor pal = palette.to(at::kFloat).contiguous();
  const float* pp = pal.data_ptr<float>();
  const int64_t* ip = ix.data_ptr<int64_t>();
  int64_t* yp = y.data_ptr<int64_t>();
  auto* xp = x.data_ptr<c10::BFloat16>();
  const uint32_t skey = mix32((uint32_t)(seed & 0xffffffff) ^ 0x9E3779B9u);
  const float kf = (float)k;
  at::parallel_for(0, B * S, 4096, [&](int64_t s0, int64_t s1) {
    for (int64_t e = s0; e < s1; ++e) {
      const int64_t b = e / S, p = e - b * S;
      const int w = (int)(p % tile), h = (int)((p / tile) % tile), d = dims == 3 ? (int)(p / tile / tile) : 0;
      const int cw = (int)((w * grid) / tile), ch = (int)((h * grid) / tile), cd = (int)((d * grid) / tile);
      const uint32_t key = mix32(skey ^ (uint32_t)ip[b]);
      const uint32_t cell = (uint32_t)((cd * grid + ch) * grid + cw);
      const int lab = (int)(mix32(key ^ mix32(cell + 0x632BE5ABu)) % (uint32_t)classes);
      yp[e] = lab;
      for (int c = 0; c < cpad; ++c) {
        float v = 0.f;
        if (c < in_ch) {
          const uint32_t base = key ^ mix32((uint32_t)(p * 8 + c) + 0x1B873593u);
          volatile float s = u24(mix32(base));
          s = s + u24(mix32(base + 0x9E3779B9u));
          s = s + u24(mix32(base + 2u * 0x9E3779B9u));
          s = s + u24(mix32(base + 3u * 0x9E3779B9u));
          volatile float t = s + -2.0f;
          volatile float n = t * kf;
          volatile float q = pp[lab * in_ch + c] + n;
          v = std::fmin(std::fmax((float)q, 0.f), 1.f);
        }
        xp[e * cpad + c] = c10::BFloat16(v);
      }
    }
  });
  return {x, y};
}

std::vector<Tensor> tile_gather(const Tensor& src, const Tensor& lab, const Tensor& idx, int64_t cpad) {
  TORCH_CHECK(src.scalar_type() == at::kByte && lab.scalar_type() == at::kByte, "uint8 dataset");
  const int64_t in_ch = src.size(-1), N = lab.size(0);
  TORCH_CHECK(in_ch >= 1 && in_ch <= 8 && cpad >= in_ch && cpad <= 8, "1 <= in_ch <= cpad <= 8");
  const Tensor ix = idx.to(at::kLong).contiguous();
  const int64_t B = ix.numel();
  const int64_t S = lab.numel() / std::max<int64_t>(1, N);
  std::vector<int64_t> ys = {B};
  for (int64_t i = 1; i < lab.dim(); ++i) ys.push_back(lab.size(i));
  Tensor y = at::empty(ys, idx.options().dtype(at::kLong));
  std::vector<int64_t> xs = ys;
  xs.push_back(cpad);
  Tensor x = at::empty(xs, src.options().dtype(at::kBFloat16));
  const Tensor sc = src.contiguous(), lc = lab.contiguous();
  const uint8_t* sp = sc.data_ptr<uint8_t>();
  const uint8_t* lp = lc.data_ptr<uint8_t>();
  const int64_t* ip = ix.data_ptr<int64_t>();
  int64_t* yp = y.data_ptr<int64_t>();
  auto* xp = x.data_ptr<c10::BFloat16>();
  for (int64_t e = 0; e < B * S; ++e) {
    const int64_t b = e / S, p = e - b * S, n = ip[b];
    const bool in_range = n >= 0 && n < N;
    const int64_t q = in_range ? n * S + p : 0;
    yp[e] = in_range ? (int64_t)lp[q] : (int64_t)-100;
    for (int c = 0; c < cpad; ++c)
      xp[e * cpad + c] = c10::BFloat16((c < in_ch && in_range) ? (float)sp[q * in_ch + c] / 255.0f : 0.f);
  }
  return {x, y};
}

}  // namespace
}  // namespace ddlpc_cpu

TORCH_LIBRARY_IMPL(ddlpc, CPU, m) {
  using namespace ddlpc_cpu;
  m.impl("conv3_fwd", &conv3_fwd);
  m.impl("conv3_wgrad", &conv3_wgrad);
  m.impl("conv3_bwd32", &conv3_bwd32);
  m.impl("reduce_rows", &reduce_rows);
  m.impl("bn_finalize", &bn_finalize);
  m.impl("bn_relu_apply", &bn_relu_apply);
  m.impl("bn_running_apply", &bn_running_apply);
  m.impl("bn_grad_coefs", &bn_grad_coefs);
  m.impl("bn_group_finalize", &bn_group_finalize);
  m.impl("bn_group_apply", &bn_group_apply);
  m.impl("bn_running_apply_all", &bn_running_apply_all);
  m.impl("bn_group_backward", &bn_group_backward);
  m.impl("bn_group_finalize_rows", &bn_group_finalize_rows);
  m.impl("bn_backward", &bn_backward);
  m.impl("convt_fwd", &convt_fwd);
  m.impl("convt_dgrad", &convt_dgrad);
  m.impl("convt_wgrad", &convt_wgrad);
  m.impl("convt_bwd_fused", &convt_bwd_fused);
  m.impl("head_ce_fwd", &head_ce_fwd);
  m.impl("head_ce_bwd", &head_ce_bwd);
  m.impl("head_ce_bn_bwd", &head_ce_bn_bwd);
  m.impl("head_ce_fwd_stats", &head_ce_fwd_stats);
  m.impl("head_wgrad_from_rows", &head_wgrad_from_rows);
  m.impl("meter_add", &meter_add);
  m.impl("head_grad_scale", &head_grad_scale);
  m.impl("head_logits", &head_logits);
  m.impl("adam_step", &adam_step);
  m.impl("adam_step_dev", &adam_step_dev);
  m.impl("weight_pack", &weight_pack);
  m.impl("codec_absmax", &codec_absmax);
  m.impl("codec_encode", &codec_encode);
  m.impl("codec_decode_sum", &codec_decode_sum);
  m.impl("bilinear_up2", &bilinear_up2);
  m.impl("bilinear_up2_bwd", &bilinear_up2_bwd);
  m.impl("to_nhwc_bf16", &to_nhwc_bf16);
  m.impl("synth_tiles", &synth_tiles);
  m.impl("tile_gather", &tile_gather);
}
