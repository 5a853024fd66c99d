// PyTorch operator registration of the hot-path stages (SURVEY 8(b) "native op layer"):
// TORCH_LIBRARY(drsa_amd, m) over the C ABI of include/drsa_amd.h, so TorchScript / C++ callers
// (torch::Dispatcher, torch.ops.drsa_amd.* from any frontend) see the same kernels the Python
// layer calls.  Host code only: every op checks its tensors, allocates outputs with the caching
// allocator and launches the libdrsa_amd kernels on the current HIP stream (no host sync, so the
// ops are graph-capturable).  A non-zero return of the C ABI becomes a c10::Error carrying
// drsa_amd_last_error().  Fake (meta) kernels for tracing are registered from Python (ops.py).
//
//   drsa_step / drsa_objective / drsa_run   cxai/xai/drsa/drsa.py:84-106, 122-155, 76-120
//   polar                                   drsa.py:201-221 (orthogonalize)
//   subspace_relevances                     cxai/xai/explain/explainer.py:206-242
//   lrp_conv_fwd / lrp_conv_bwd / lrp_linear_fwd / lrp_linear_bwd / projection_fwd / projection_bwd
//                                           the zennit rule passes attribute.py:98-107 drives
//   heatmap_sort                            explainer.py:99-123, 151-176
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <initializer_list>
#include <tuple>

#include "drsa_amd.h"

namespace {

using at::Tensor;

void* cur_stream() { return reinterpret_cast<void*>(c10::hip::getCurrentHIPStream().stream()); }

void check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, ": ", drsa_amd_last_error(), " (code ", rc, ")");
}

void need(const Tensor& t, const char* name, at::ScalarType dt = at::kFloat) {
  TORCH_CHECK(t.is_cuda(), "drsa_amd: ", name, " must be a GPU tensor (there is no CPU kernel)");
  TORCH_CHECK(t.scalar_type() == dt, "drsa_amd: ", name, " must be ", dt, ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), "drsa_amd: ", name, " must be contiguous");
}

// Every op runs on the device of its first tensor argument (guard below: the current stream is
// that device's) and refuses tensors on another device instead of queueing kernels that would
// touch another GPU's memory.
void same_device(const Tensor& ref, std::initializer_list<const Tensor*> ts) {
  for (const Tensor* t : ts)
    TORCH_CHECK(!t->defined() || t->numel() == 0 || t->device() == ref.device(),
                "drsa_amd: all tensor arguments must be on ", ref.device(), ", got one on ", t->device());
}
void same_device(const Tensor& ref, const c10::optional<Tensor>& t) {
  if (t.has_value()) same_device(ref, {&*t});
}
#define DRSA_GUARD(t) const at::OptionalDeviceGuard device_guard_(at::device_of(t))

template <class T = float>
const T* cptr(const c10::optional<Tensor>& t) { return t.has_value() ? t->data_ptr<T>() : nullptr; }

struct Ws {   // DRSA workspace (DrsaWorkspace in xai/drsa/drsa.py)
  Tensor buf, counter, f;
  Ws(int64_t N, int64_t d, int64_t K, const at::TensorOptions& o) {
    const size_t nb = drsa_amd_drsa_workspace_bytes(N, (int)d, (int)K);
    TORCH_CHECK(nb > 0, "drsa_amd: unsupported DRSA problem N=", N, " d=", d, " K=", K);
    buf = at::empty({(int64_t)nb}, o.dtype(at::kByte));
    counter = at::zeros({4}, o.dtype(at::kInt));
    f = at::empty({1}, o.dtype(at::kFloat));
  }
};

void check_problem(const Tensor& A, const Tensor& C, const Tensor& U, int64_t K) {
  need(A, "activation_vecs"), need(C, "context_vecs"), need(U, "U");
  same_device(A, {&C, &U});
  TORCH_CHECK(A.dim() == 2 && A.sizes() == C.sizes(), "drsa_amd: activation and context vectors must be [N, d]");
  const int64_t d = A.size(1);
  TORCH_CHECK(U.dim() == 2 && U.size(0) == d && U.size(1) == d, "drsa_amd: U must be [", d, ", ", d, "]");
  TORCH_CHECK(K > 0 && d % K == 0, "drsa_amd: num_concepts must be a positive divisor of d");
}

std::tuple<Tensor, Tensor> drsa_step(const Tensor& A, const Tensor& C, const Tensor& U, int64_t K) {
  DRSA_GUARD(A);
  check_problem(A, C, U, K);
  Ws ws(A.size(0), A.size(1), K, A.options());
  Tensor Un = at::empty_like(U);
  check(drsa_amd_drsa_step(A.data_ptr<float>(), C.data_ptr<float>(), A.size(0), (int)A.size(1), (int)K,
                           U.data_ptr<float>(), Un.data_ptr<float>(), ws.f.data_ptr<float>(), ws.buf.data_ptr(),
                           ws.buf.numel(), cur_stream()),
        "drsa_step");
  return {Un, ws.f.reshape({})};
}

Tensor drsa_objective(const Tensor& A, const Tensor& C, const Tensor& U, int64_t K) {
  DRSA_GUARD(A);
  check_problem(A, C, U, K);
  Ws ws(A.size(0), A.size(1), K, A.options());
  check(drsa_amd_drsa_objective(A.data_ptr<float>(), C.data_ptr<float>(), A.size(0), (int)A.size(1), (int)K,
                                U.data_ptr<float>(), ws.f.data_ptr<float>(), ws.buf.data_ptr(), ws.buf.numel(),
                                cur_stream()),
        "drsa_objective");
  return ws.f.reshape({});
}

std::tuple<Tensor, Tensor> drsa_run_16(const Tensor& A, const Tensor& C, const Tensor& U0, int64_t K, int64_t steps) {
  // C5 bf16 / fp16 activation and context rows: the one-problem form of drsa_amd_drsa_run_multi
  // (U-projection GEMM on bf16 / fp16 MFMA, fp32 accumulation and polar), as drsa_run_joint does
  const at::ScalarType dt = A.scalar_type();
  need(A, "activation_vecs", dt), need(C, "context_vecs", dt), need(U0, "U");
  same_device(A, {&C, &U0});
  TORCH_CHECK(A.dim() == 2 && A.sizes() == C.sizes(), "drsa_amd: activation and context vectors must be [N, d]");
  const int64_t d = A.size(1);
  TORCH_CHECK(U0.dim() == 2 && U0.size(0) == d && U0.size(1) == d, "drsa_amd: U must be [", d, ", ", d, "]");
  TORCH_CHECK(K > 0 && d % K == 0, "drsa_amd: num_concepts must be a positive divisor of d");
  TORCH_CHECK(steps >= 0, "drsa_amd: steps must be >= 0");
  Ws ws(A.size(0), d, K, A.options());
  Tensor U = U0.clone();
  Tensor Ut = at::empty_like(U);
  Tensor traj = at::empty({steps + 1}, U0.options());
  drsa_amd_problem_t p{};
  p.A = static_cast<const float*>(A.data_ptr());
  p.C = static_cast<const float*>(C.data_ptr());
  p.N = A.size(0);
  p.d = (int)d;
  p.K = (int)K;
  p.U_io = U.data_ptr<float>();
  p.U_tmp = Ut.data_ptr<float>();
  p.f_traj = traj.data_ptr<float>();
  p.counter = ws.counter.data_ptr<int>();
  p.ws = ws.buf.data_ptr();
  p.ws_size = ws.buf.numel();
  p.dtype = dt == at::kBFloat16 ? 1 : 2;
  void* s = cur_stream();
  check(drsa_amd_drsa_run_multi(1, &p, (int)steps, s != nullptr ? 1 : 0, s), "drsa_run (16-bit rows)");
  return {U, traj};
}

std::tuple<Tensor, Tensor> drsa_run(const Tensor& A, const Tensor& C, const Tensor& U0, int64_t K, int64_t steps) {
  DRSA_GUARD(A);
  if (A.scalar_type() == at::kBFloat16 || A.scalar_type() == at::kHalf) return drsa_run_16(A, C, U0, K, steps);
  check_problem(A, C, U0, K);
  TORCH_CHECK(steps >= 0, "drsa_amd: steps must be >= 0");
  Ws ws(A.size(0), A.size(1), K, A.options());
  Tensor U = U0.clone();
  Tensor Ut = at::empty_like(U);
  Tensor traj = at::empty({steps + 1}, A.options());
  void* s = cur_stream();
  // the whole loop as one captured hipGraph on a non-default stream (the library records the
  // plain launch sequence while a caller's capture is active)
  check(drsa_amd_drsa_run(A.data_ptr<float>(), C.data_ptr<float>(), A.size(0), (int)A.size(1), (int)K,
                          U.data_ptr<float>(), Ut.data_ptr<float>(), (int)steps, traj.data_ptr<float>(),
                          ws.counter.data_ptr<int>(), ws.buf.data_ptr(), ws.buf.numel(), s != nullptr ? 1 : 0, s),
        "drsa_run");
  return {U, traj};
}

Tensor polar(const Tensor& V_) {
  DRSA_GUARD(V_);
  Tensor V = V_.contiguous();
  need(V, "V");
  TORCH_CHECK(V.dim() == 2 && V.size(0) == V.size(1), "drsa_amd: polar needs a square matrix");
  Tensor out = at::empty_like(V);
  check(drsa_amd_polar(V.data_ptr<float>(), (int)V.size(0), out.data_ptr<float>(), nullptr, cur_stream()), "polar");
  return out;
}

Tensor subspace_relevances(const Tensor& act, const Tensor& ctx, const Tensor& U_, int64_t K) {
  DRSA_GUARD(act);
  TORCH_CHECK(act.dim() < 4 || ctx.dim() < 4, "drsa_amd: act and ctx must be [batch, N, d] or [N, d]");
  TORCH_CHECK(act.is_cuda(), "drsa_amd: act must be a GPU tensor (there is no CPU kernel)");
  same_device(act, {&ctx, &U_});
  // explainer.py:168-180 semantics: any float dtype / layout, computed in fp32
  Tensor a = (act.dim() == 3 ? act : act.unsqueeze(0)).to(at::kFloat).contiguous();
  Tensor c = (ctx.dim() == 3 ? ctx : ctx.unsqueeze(0)).to(at::kFloat).contiguous();
  Tensor U = U_.to(at::kFloat).contiguous();
  need(a, "act"), need(c, "ctx"), need(U, "U");
  TORCH_CHECK(a.dim() == 3 && c.sizes() == a.sizes(), "drsa_amd: act and ctx must have one shape [b, N, d]");
  const int64_t b = a.size(0), N = a.size(1), d = a.size(2);
  TORCH_CHECK(U.dim() == 2 && U.size(0) == d && U.size(1) == d, "drsa_amd: U must be [d, d]");
  TORCH_CHECK(K > 0 && d % K == 0, "drsa_amd: num_concepts must divide d");
  Tensor out = at::empty({b, K}, a.options());
  const size_t nb = drsa_amd_subspace_relevances_workspace_bytes(b, N, (int)d, (int)K);
  TORCH_CHECK(nb > 0, "drsa_amd: unsupported subspace_relevances problem b=", b, " N=", N, " d=", d, " K=", K);
  Tensor ws = at::empty({(int64_t)nb}, a.options().dtype(at::kByte));
  check(drsa_amd_subspace_relevances(a.data_ptr<float>(), c.data_ptr<float>(), b, N, (int)d, (int)K,
                                     U.data_ptr<float>(), out.data_ptr<float>(), ws.data_ptr(), nb, cur_stream()),
        "subspace_relevances");
  return out;
}

std::tuple<Tensor, Tensor, Tensor> lrp_conv_fwd(const Tensor& x, const Tensor& wts, const Tensor& bias3,
                                                const c10::optional<Tensor>& den_map, int64_t cout, int64_t ng,
                                                bool pool) {
  DRSA_GUARD(x);
  need(x, "x"), need(wts, "wts"), need(bias3, "bias3");
  same_device(x, {&wts, &bias3}), same_device(x, den_map);
  TORCH_CHECK(x.dim() == 4, "drsa_amd: x must be [B, C, H, W]");
  const int64_t B = x.size(0), cin = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W;
  Tensor y = at::empty({B, cout, Ho, Wo}, x.options());
  Tensor amax = pool ? at::empty({B, cout, Ho, Wo}, x.options().dtype(at::kByte)) : at::empty({0}, x.options().dtype(at::kByte));
  Tensor den = at::empty({B, cout, Ho, Wo}, x.options());
  check(drsa_amd_conv_fwd(x.data_ptr<float>(), wts.data_ptr<float>(), bias3.data_ptr<float>(), cptr(den_map),
                          y.data_ptr<float>(), pool ? amax.data_ptr<uint8_t>() : nullptr, den.data_ptr<float>(),
                          (int)B, (int)cin, (int)cout, (int)H, (int)W, (int)ng, pool ? 1 : 0, cur_stream()),
        "lrp_conv_fwd");
  return {y, amax, den};
}

Tensor lrp_conv_bwd(const Tensor& g, const c10::optional<Tensor>& amax, const Tensor& wts,
                    const c10::optional<Tensor>& x, const c10::optional<Tensor>& den, int64_t cin, int64_t H, int64_t W,
                    int64_t clones, int64_t ng, int64_t xmode, int64_t post, double eps) {
  DRSA_GUARD(g);
  need(g, "g"), need(wts, "wts");
  same_device(g, {&wts}), same_device(g, amax), same_device(g, x), same_device(g, den);
  const int64_t Bq = g.size(0), cout = g.size(1);
  Tensor out = at::empty({Bq, cin, H, W}, g.options());
  check(drsa_amd_conv_bwd(g.data_ptr<float>(), cptr<uint8_t>(amax), wts.data_ptr<float>(), cptr(x), cptr(den),
                          out.data_ptr<float>(), (int)Bq, (int)clones, (int)cout, (int)cin, (int)H, (int)W, (int)ng,
                          (int)xmode, (int)post, (float)eps, cur_stream()),
        "lrp_conv_bwd");
  return out;
}

std::tuple<Tensor, Tensor> lrp_linear_fwd(const Tensor& x, const Tensor& Wt, const c10::optional<Tensor>& b,
                                          bool relu) {
  DRSA_GUARD(x);
  need(x, "x"), need(Wt, "W");
  same_device(x, {&Wt}), same_device(x, b);
  const int64_t M = x.size(0), K = x.size(1), N = Wt.size(0);
  Tensor z = at::empty({M, N}, x.options());
  Tensor a = relu ? at::empty({M, N}, x.options()) : at::empty({0}, x.options());
  check(drsa_amd_linear_fwd(x.data_ptr<float>(), Wt.data_ptr<float>(), cptr(b), z.data_ptr<float>(),
                            relu ? a.data_ptr<float>() : nullptr, (int)M, (int)N, (int)K, cur_stream()),
        "lrp_linear_fwd");
  return {z, a};
}

Tensor lrp_linear_bwd(const c10::optional<Tensor>& R, const c10::optional<Tensor>& cls, bool one_hot, const Tensor& z,
                      bool relu_mask, bool rule_eps, double eps, const Tensor& Wt, const Tensor& x, int64_t xmode,
                      const c10::optional<Tensor>& den, int64_t post, double eps_post) {
  DRSA_GUARD(z);
  need(z, "z"), need(Wt, "W"), need(x, "x");
  same_device(z, {&Wt, &x}), same_device(z, R), same_device(z, cls), same_device(z, den);
  const int64_t M = z.size(0), Nout = z.size(1), Kin = Wt.size(1);
  Tensor out = at::empty({M, Kin}, z.options());
  check(drsa_amd_linear_bwd(cptr(R), cptr<int>(cls), one_hot ? 1 : 0, z.data_ptr<float>(), relu_mask ? 1 : 0,
                            rule_eps ? 1 : 0, (float)eps, Wt.data_ptr<float>(), x.data_ptr<float>(), (int)xmode,
                            cptr(den), (int)post, (float)eps_post, out.data_ptr<float>(), (int)M, (int)Nout, (int)Kin,
                            cur_stream()),
        "lrp_linear_bwd");
  return out;
}

Tensor residual(const Tensor& U) {   // P = U U^T - I (drsa_amd_projection_residual)
  Tensor P = at::empty_like(U);
  check(drsa_amd_projection_residual(U.data_ptr<float>(), (int)U.size(0), P.data_ptr<float>(), cur_stream()),
        "projection_residual");
  return P;
}

std::tuple<Tensor, Tensor> projection_fwd(const Tensor& a, const Tensor& U, bool pool) {
  DRSA_GUARD(a);
  need(a, "a"), need(U, "U");
  same_device(a, {&U});
  const int64_t B = a.size(0), D = a.size(1), H = a.size(2), W = a.size(3);
  Tensor P = residual(U);
  if (pool) {
    Tensor y = at::empty({B, D, H / 2, W / 2}, a.options());
    Tensor amax = at::empty({B, D, H / 2, W / 2}, a.options().dtype(at::kByte));
    check(drsa_amd_projection_fwd(a.data_ptr<float>(), U.data_ptr<float>(), P.data_ptr<float>(), nullptr, nullptr,
                                  y.data_ptr<float>(), amax.data_ptr<uint8_t>(), (int)B, (int)D, (int)H, (int)W, 1,
                                  cur_stream()),
          "projection_fwd");
    return {y, amax};
  }
  Tensor y = at::empty_like(a);
  check(drsa_amd_projection_fwd(a.data_ptr<float>(), U.data_ptr<float>(), P.data_ptr<float>(), nullptr,
                                y.data_ptr<float>(), nullptr, nullptr, (int)B, (int)D, (int)H, (int)W, 0, cur_stream()),
        "projection_fwd");
  return {y, at::empty({0}, a.options().dtype(at::kByte))};
}

Tensor projection_bwd(const Tensor& g, const c10::optional<Tensor>& amax, const Tensor& a,
                      const c10::optional<Tensor>& den, const Tensor& U, int64_t K, double eps_proj, double eps_den,
                      bool fanout) {
  DRSA_GUARD(a);
  need(g, "g"), need(a, "a"), need(U, "U");
  same_device(a, {&g, &U}), same_device(a, amax), same_device(a, den);
  const int64_t B = a.size(0), D = a.size(1), H = a.size(2), W = a.size(3);
  const int64_t nq = fanout ? K + 1 : 1;
  Tensor G = at::empty({B * nq, D, H, W}, a.options());
  Tensor P = residual(U);
  check(drsa_amd_projection_bwd(g.data_ptr<float>(), cptr<uint8_t>(amax), nullptr, nullptr, a.data_ptr<float>(),
                                cptr(den), U.data_ptr<float>(), P.data_ptr<float>(), G.data_ptr<float>(), (int)B, (int)D,
                                (int)H, (int)W, (int)K, (float)eps_proj, (float)eps_den, fanout ? 1 : 0, cur_stream()),
        "projection_bwd");
  return G;
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> heatmap_sort(const Tensor& hm, int64_t K, bool std_from_sum) {
  DRSA_GUARD(hm);
  need(hm, "hm");
  const int64_t H = hm.size(-2), W = hm.size(-1);
  const int64_t B = hm.numel() / ((std_from_sum ? K : K + 1) * H * W);
  Tensor std_ = at::empty({B, 1, H, W}, hm.options());
  Tensor std_rel = at::empty({B}, hm.options());
  Tensor sub = at::empty({B, K, H, W}, hm.options());
  Tensor rel = at::empty({B, K}, hm.options());
  Tensor mask = at::empty({B, K}, hm.options().dtype(at::kLong));
  check(drsa_amd_heatmap_sort(hm.data_ptr<float>(), (int)B, (int)K, (int)(H * W), std_from_sum ? 1 : 0,
                              std_.data_ptr<float>(), std_rel.data_ptr<float>(), sub.data_ptr<float>(),
                              rel.data_ptr<float>(), mask.data_ptr<int64_t>(), cur_stream()),
        "heatmap_sort");
  return {std_, std_rel, sub, rel, mask};
}

}  // namespace

TORCH_LIBRARY(drsa_amd, m) {
  m.def("drsa_step(Tensor A, Tensor C, Tensor U, int K) -> (Tensor, Tensor)");
  m.def("drsa_objective(Tensor A, Tensor C, Tensor U, int K) -> Tensor");
  m.def("drsa_run(Tensor A, Tensor C, Tensor U0, int K, int steps) -> (Tensor, Tensor)");
  m.def("polar(Tensor V) -> Tensor");
  m.def("subspace_relevances(Tensor act, Tensor ctx, Tensor U, int K) -> Tensor");
  m.def("lrp_conv_fwd(Tensor x, Tensor wts, Tensor bias3, Tensor? den_map, int cout, int ng, bool pool) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("lrp_conv_bwd(Tensor g, Tensor? amax, Tensor wts, Tensor? x, Tensor? den, int cin, int H, int W, "
        "int clones, int ng, int xmode, int post, float eps) -> Tensor");
  m.def("lrp_linear_fwd(Tensor x, Tensor W, Tensor? b, bool relu) -> (Tensor, Tensor)");
  m.def("lrp_linear_bwd(Tensor? R, Tensor? cls, bool one_hot, Tensor z, bool relu_mask, bool rule_eps, float eps, "
        "Tensor W, Tensor x, int xmode, Tensor? den, int post, float eps_post) -> Tensor");
  m.def("projection_fwd(Tensor a, Tensor U, bool pool) -> (Tensor, Tensor)");
  m.def("projection_bwd(Tensor g, Tensor? amax, Tensor a, Tensor? den, Tensor U, int K, float eps_proj, "
        "float eps_den, bool fanout) -> Tensor");
  m.def("heatmap_sort(Tensor hm, int K, bool std_from_sum=False) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(drsa_amd, CUDA, m) {
  m.impl("drsa_step", &drsa_step);
  m.impl("drsa_objective", &drsa_objective);
  m.impl("drsa_run", &drsa_run);
  m.impl("polar", &polar);
  m.impl("subspace_relevances", &subspace_relevances);
  m.impl("lrp_conv_fwd", &lrp_conv_fwd);
  m.impl("lrp_conv_bwd", &lrp_conv_bwd);
  m.impl("lrp_linear_fwd", &lrp_linear_fwd);
  m.impl("lrp_linear_bwd", &lrp_linear_bwd);
  m.impl("projection_fwd", &projection_fwd);
  m.impl("projection_bwd", &projection_bwd);
  m.impl("heatmap_sort", &heatmap_sort);
}
