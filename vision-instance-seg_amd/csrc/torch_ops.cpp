// torch.ops.visionseg.* -- the operator surface of SURVEY §8(b) registered with
// TORCH_LIBRARY over the C ABI of libvisionseg_hip.so (include/visionseg.h).
//
// Contract (§8(b) "Operator C-ABI"): ATen tensors in, outputs allocated here through the
// caching allocator (the caller owns them), launches on the current HIP stream of the
// inputs' device, errors raised with TORCH_CHECK (-> Python RuntimeError), no host sync
// inside an op (msda_*: spatial_shapes / level_start_index are read on the host; pass CPU
// int64 tensors -- a device tensor costs one device->host copy, as the upstream extension's
// callers do with `.tolist()`), no global state.  The autograd wrappers stay in Python
// (visionseg/ops.py), as the upstream `MSDeformAttnFunction` wraps its extension.
// There is no CPU kernel: a CPU tensor is refused (no fallback path exists).
//
// Host-only C++ (g++), linked against libvisionseg_hip.so; the kernels live in csrc/*.hip.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <string>
#include <vector>

#include "../../include/visionseg.h"

namespace {

void vs_ok(int rc, const char* what) {
  TORCH_CHECK(rc == VS_OK, "visionseg ", what, " failed (status ", rc, "): ", vs_last_error());
}

void* cur_stream(const at::Tensor& t) {
  return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

int dcode(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return VS_F32;
  if (t.scalar_type() == at::kBFloat16) return VS_BF16;
  TORCH_CHECK(false, "visionseg kernels take float32 or bfloat16 activations, got ", t.scalar_type());
  return -1;
}

void on_device(std::initializer_list<const at::Tensor*> ts) {
  for (const at::Tensor* t : ts)
    TORCH_CHECK(t->is_cuda(), "visionseg ops run only on a HIP device (no CPU fallback); got a tensor on ",
                t->device());
}

int as_int(int64_t v, const char* what) {
  TORCH_CHECK(v >= 0 && v <= INT32_MAX, what, " out of range: ", v);
  return (int)v;
}

// spatial_shapes [L, 2] / level_start_index [L] int64 -> host vectors (the C ABI reads them
// on the host: they size the launch)
std::vector<int64_t> host_i64(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.scalar_type() == at::kLong, what, " must be int64");
  at::Tensor h = t.device().is_cpu() ? t.contiguous() : t.to(at::kCPU).contiguous();
  return std::vector<int64_t>(h.data_ptr<int64_t>(), h.data_ptr<int64_t>() + h.numel());
}

// ---- a8: MSDeformAttn sampling (upstream MultiScaleDeformableAttention.ms_deform_attn_*)
struct MsdaDims {
  int64_t B, S, H, D, Q, L, P;
};

// one shape check for both directions: value [B, S, heads, 32], sampling_loc [B, Q, heads, L,
// P, 2] f32, attn_weight [B, Q, heads, L, P] f32, L levels of shapes / starts
MsdaDims check_msda(const at::Tensor& value, const std::vector<int64_t>& sh, const std::vector<int64_t>& st,
                    const at::Tensor& loc, const at::Tensor& aw) {
  TORCH_CHECK(value.dim() == 4, "value must be [B, S, heads, 32]");
  TORCH_CHECK(loc.dim() == 6 && loc.size(5) == 2, "sampling_loc must be [B, Q, heads, L, P, 2]");
  TORCH_CHECK(loc.scalar_type() == at::kFloat && aw.scalar_type() == at::kFloat,
              "sampling_loc / attn_weight must be float32");
  MsdaDims d{value.size(0), value.size(1), value.size(2), value.size(3), loc.size(1), loc.size(3), loc.size(4)};
  TORCH_CHECK((int64_t)sh.size() == 2 * d.L && (int64_t)st.size() == d.L,
              "spatial_shapes / level_start_index do not have ", d.L, " levels");
  TORCH_CHECK(loc.size(0) == d.B && loc.size(2) == d.H, "sampling_loc batch/heads do not match value");
  TORCH_CHECK(aw.sizes() == at::IntArrayRef({d.B, d.Q, d.H, d.L, d.P}), "attn_weight must be [B, Q, heads, L, P]");
  return d;
}

at::Tensor msda_fwd(const at::Tensor& value, const at::Tensor& spatial_shapes, const at::Tensor& level_start_index,
                    const at::Tensor& sampling_loc, const at::Tensor& attn_weight, int64_t im2col_step) {
  (void)im2col_step;  // the kernel tiles by query groups, not im2col steps
  on_device({&value, &sampling_loc, &attn_weight});
  const auto sh = host_i64(spatial_shapes, "spatial_shapes");
  const auto st = host_i64(level_start_index, "level_start_index");
  at::Tensor v = value.contiguous(), loc = sampling_loc.contiguous(), aw = attn_weight.contiguous();
  const MsdaDims d = check_msda(v, sh, st, loc, aw);
  at::Tensor out = at::empty({d.B, d.Q, d.H * d.D}, v.options());
  vs_ok(vs_msda_forward(dcode(v), v.data_ptr(), sh.data(), st.data(), loc.data_ptr<float>(), aw.data_ptr<float>(),
                        out.data_ptr(), as_int(d.B, "batch"), as_int(d.S, "S"), as_int(d.H, "heads"),
                        as_int(d.D, "channels"), as_int(d.L, "levels"), as_int(d.Q, "queries"), as_int(d.P, "points"),
                        cur_stream(v)),
        "msda_fwd");
  return out;
}

// -> (grad_value in value's dtype -- or the f32 accumulator itself with f32_grad_value --,
//     grad_sampling_loc f32, grad_attn_weight f32)
std::tuple<at::Tensor, at::Tensor, at::Tensor> msda_bwd(const at::Tensor& value, const at::Tensor& spatial_shapes,
                                                        const at::Tensor& level_start_index,
                                                        const at::Tensor& sampling_loc, const at::Tensor& attn_weight,
                                                        const at::Tensor& grad_output, int64_t im2col_step,
                                                        bool f32_grad_value) {
  (void)im2col_step;
  on_device({&value, &sampling_loc, &attn_weight, &grad_output});
  const auto sh = host_i64(spatial_shapes, "spatial_shapes");
  const auto st = host_i64(level_start_index, "level_start_index");
  at::Tensor v = value.contiguous(), loc = sampling_loc.contiguous(), aw = attn_weight.contiguous();
  const MsdaDims d = check_msda(v, sh, st, loc, aw);
  TORCH_CHECK(grad_output.numel() == d.B * d.Q * d.H * d.D && grad_output.dim() >= 2 && grad_output.size(0) == d.B &&
                  grad_output.size(1) == d.Q,
              "grad_output must be [B, Q, heads*32]");
  at::Tensor g = grad_output.to(v.scalar_type()).contiguous();
  // grad_value accumulates in f32 (float atomics), then takes value's dtype
  at::Tensor gv = at::empty({d.B, d.S, d.H, d.D}, v.options().dtype(at::kFloat));
  at::Tensor gl = at::empty_like(loc), ga = at::empty_like(aw);
  // workspace: reserved by the C ABI (0 bytes since round 6; csrc/msda.hip)
  const long long wsb = vs_msda_backward_workspace_bytes(as_int(d.B, "batch"), as_int(d.Q, "queries"),
                                                         as_int(d.H, "heads"), as_int(d.L, "levels"),
                                                         as_int(d.P, "points"));
  TORCH_CHECK(wsb >= 0, "msda_bwd: bad sizes");
  at::Tensor ws = at::empty({wsb}, v.options().dtype(at::kByte));
  vs_ok(vs_msda_backward_ex(dcode(v), v.data_ptr(), sh.data(), st.data(), loc.data_ptr<float>(),
                            aw.data_ptr<float>(), g.data_ptr(), gv.data_ptr<float>(), gl.data_ptr<float>(),
                            ga.data_ptr<float>(), ws.data_ptr(), as_int(d.B, "batch"), as_int(d.S, "S"),
                            as_int(d.H, "heads"), as_int(d.D, "channels"), as_int(d.L, "levels"),
                            as_int(d.Q, "queries"), as_int(d.P, "points"), cur_stream(v)),
        "msda_bwd");
  return {(v.scalar_type() == at::kFloat || f32_grad_value) ? gv : gv.to(v.scalar_type()), gl, ga};
}

// ---- a2: pad + roll + window partition (and its exact inverse)
int64_t padded(int64_t n, int64_t ws) { return n + (ws - n % ws) % ws; }

at::Tensor swin_window_fwd(const at::Tensor& x, int64_t window, int64_t shift) {
  on_device({&x});
  TORCH_CHECK(x.dim() == 4, "x must be [B, H, W, C]");
  TORCH_CHECK(window > 0 && shift >= 0 && shift < window, "bad window / shift");
  at::Tensor xc = x.contiguous();
  const int64_t B = xc.size(0), H = xc.size(1), W = xc.size(2), C = xc.size(3);
  const int64_t nw = (padded(H, window) / window) * (padded(W, window) / window);
  at::Tensor out = at::empty({B * nw, window * window, C}, xc.options());
  vs_ok(vs_window_partition(xc.data_ptr(), out.data_ptr(), (int)xc.element_size(), as_int(B, "batch"),
                            as_int(H, "height"), as_int(W, "width"), as_int(C, "channels"), (int)window, (int)shift,
                            cur_stream(xc)),
        "swin_window_fwd");
  return out;
}

at::Tensor swin_window_bwd(const at::Tensor& windows, int64_t batch, int64_t height, int64_t width, int64_t window,
                           int64_t shift) {
  on_device({&windows});
  TORCH_CHECK(windows.dim() == 3 && windows.size(1) == window * window, "windows must be [B*nW, window^2, C]");
  const int64_t nw = (padded(height, window) / window) * (padded(width, window) / window);
  TORCH_CHECK(windows.size(0) == batch * nw, "windows hold ", windows.size(0), " windows, expected ", batch * nw);
  at::Tensor wc = windows.contiguous();
  const int64_t C = wc.size(2);
  at::Tensor out = at::empty({batch, height, width, C}, wc.options());
  vs_ok(vs_window_reverse(wc.data_ptr(), out.data_ptr(), (int)wc.element_size(), as_int(batch, "batch"),
                          as_int(height, "height"), as_int(width, "width"), as_int(C, "channels"), (int)window,
                          (int)shift, cur_stream(wc)),
        "swin_window_bwd");
  return out;
}

// ---- a3/a4/a5: window attention core (qkv = the fused q;k;v Linear output per window)
void check_qkv(const at::Tensor& qkv, int64_t heads, int64_t window) {
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(1) == window * window && qkv.size(2) == 3 * heads * 32,
              "qkv must be [B*nW, window^2, 3*heads*32]");
}

std::tuple<at::Tensor, at::Tensor> win_attn_fwd(const at::Tensor& qkv, const at::Tensor& rel_table, int64_t heads,
                                                int64_t window, int64_t shift, int64_t nwin_h, int64_t nwin_w,
                                                double scale, bool fp8) {
  on_device({&qkv, &rel_table});
  check_qkv(qkv, heads, window);
  at::Tensor q = qkv.contiguous(), table = rel_table.to(at::kFloat).contiguous();
  TORCH_CHECK(table.numel() == (2 * window - 1) * (2 * window - 1) * heads, "rel_table must be [(2ws-1)^2, heads]");
  const int64_t Bw = q.size(0), N = q.size(1);
  at::Tensor out = at::empty({Bw, N, heads * 32}, q.options());
  at::Tensor lse = at::empty({Bw, heads, N}, q.options().dtype(at::kFloat));
  if (fp8) {
    TORCH_CHECK(q.scalar_type() == at::kBFloat16 && N <= 160, "fp8 window attention needs bf16 qkv and window^2 <= 160");
    vs_ok(vs_window_attn_forward_fp8(q.data_ptr(), table.data_ptr<float>(), out.data_ptr(), lse.data_ptr<float>(),
                                     as_int(Bw, "windows"), (int)heads, (int)window, (int)shift, (int)nwin_h,
                                     (int)nwin_w, (float)scale, cur_stream(q)),
          "win_attn_fwd (fp8)");
  } else {
    vs_ok(vs_window_attn_forward(dcode(q), q.data_ptr(), table.data_ptr<float>(), out.data_ptr(),
                                 lse.data_ptr<float>(), as_int(Bw, "windows"), (int)heads, (int)window, (int)shift,
                                 (int)nwin_h, (int)nwin_w, (float)scale, cur_stream(q)),
          "win_attn_fwd");
  }
  return {out, lse};
}

// -> (grad_qkv, grad_rel_table [(2ws-1)^2, heads] f32)
std::tuple<at::Tensor, at::Tensor> win_attn_bwd(const at::Tensor& qkv, const at::Tensor& rel_table,
                                                const at::Tensor& out, const at::Tensor& lse,
                                                const at::Tensor& grad_out, int64_t heads, int64_t window,
                                                int64_t shift, int64_t nwin_h, int64_t nwin_w, double scale,
                                                bool fp8, bool table_partials) {
  on_device({&qkv, &rel_table, &out, &lse, &grad_out});
  check_qkv(qkv, heads, window);
  at::Tensor q = qkv.contiguous(), table = rel_table.to(at::kFloat).contiguous();
  at::Tensor o = out.contiguous(), l = lse.contiguous(), g = grad_out.to(q.scalar_type()).contiguous();
  const int64_t Bw = q.size(0), N = q.size(1), T2 = (2 * window - 1) * (2 * window - 1);
  TORCH_CHECK(o.sizes() == at::IntArrayRef({Bw, N, heads * 32}) && g.sizes() == o.sizes(),
              "out / grad_out must be [B*nW, window^2, heads*32]");
  TORCH_CHECK(l.scalar_type() == at::kFloat && l.sizes() == at::IntArrayRef({Bw, heads, N}),
              "lse must be float32 [B*nW, heads, window^2]");
  TORCH_CHECK(table.numel() == T2 * heads, "rel_table must be [(2ws-1)^2, heads]");
  at::Tensor gqkv = at::empty_like(q);
  at::Tensor part = at::empty({Bw, heads, T2}, q.options().dtype(at::kFloat));
  if (fp8) {
    vs_ok(vs_window_attn_backward_fp8(q.data_ptr(), table.data_ptr<float>(), o.data_ptr(), l.data_ptr<float>(),
                                      g.data_ptr(), gqkv.data_ptr(), part.data_ptr<float>(), as_int(Bw, "windows"),
                                      (int)heads, (int)window, (int)shift, (int)nwin_h, (int)nwin_w, (float)scale,
                                      cur_stream(q)),
          "win_attn_bwd (fp8)");
  } else {
    vs_ok(vs_window_attn_backward(dcode(q), q.data_ptr(), table.data_ptr<float>(), o.data_ptr(), l.data_ptr<float>(),
                                  g.data_ptr(), gqkv.data_ptr(), part.data_ptr<float>(), as_int(Bw, "windows"),
                                  (int)heads, (int)window, (int)shift, (int)nwin_h, (int)nwin_w, (float)scale,
                                  cur_stream(q)),
          "win_attn_bwd");
  }
  // per-window partial bias gradients summed in a fixed order (deterministic); or the
  // partials themselves [Bw, heads, (2ws-1)^2] (table_partials)
  if (table_partials) return {gqkv, part};
  return {gqkv, part.sum(0).t().contiguous()};
}

// image-layout window attention (the window reverse folded in): out / grad_out
// [B, height, width, heads*32]; qkv, lse, grad_qkv in the window layout
std::tuple<at::Tensor, at::Tensor> win_attn_fwd_img(const at::Tensor& qkv, const at::Tensor& rel_table, int64_t heads,
                                                    int64_t window, int64_t shift, int64_t nwin_h, int64_t nwin_w,
                                                    int64_t height, int64_t width, double scale, bool fp8) {
  on_device({&qkv, &rel_table});
  check_qkv(qkv, heads, window);
  at::Tensor q = qkv.contiguous(), table = rel_table.to(at::kFloat).contiguous();
  TORCH_CHECK(table.numel() == (2 * window - 1) * (2 * window - 1) * heads, "rel_table must be [(2ws-1)^2, heads]");
  const int64_t Bw = q.size(0), N = q.size(1), nw = nwin_h * nwin_w;
  TORCH_CHECK(nw > 0 && Bw % nw == 0, "num_windows must be a multiple of nwin_h * nwin_w");
  at::Tensor out = at::empty({Bw / nw, height, width, heads * 32}, q.options());
  at::Tensor lse = at::empty({Bw, heads, N}, q.options().dtype(at::kFloat));
  vs_ok(vs_window_attn_forward_image(dcode(q), fp8 ? 1 : 0, q.data_ptr(), table.data_ptr<float>(), out.data_ptr(),
                                     lse.data_ptr<float>(), as_int(Bw, "windows"), (int)heads, (int)window,
                                     (int)shift, (int)nwin_h, (int)nwin_w, as_int(height, "height"),
                                     as_int(width, "width"), (float)scale, cur_stream(q)),
        "win_attn_fwd_img");
  return {out, lse};
}

// -> (grad_qkv [window layout], grad_rel_table partials [Bw, heads, (2ws-1)^2] f32)
std::tuple<at::Tensor, at::Tensor> win_attn_bwd_img(const at::Tensor& qkv, const at::Tensor& rel_table,
                                                    const at::Tensor& out, const at::Tensor& lse,
                                                    const at::Tensor& grad_out, int64_t heads, int64_t window,
                                                    int64_t shift, int64_t nwin_h, int64_t nwin_w, int64_t height,
                                                    int64_t width, double scale, bool fp8) {
  on_device({&qkv, &rel_table, &out, &lse, &grad_out});
  check_qkv(qkv, heads, window);
  at::Tensor q = qkv.contiguous(), table = rel_table.to(at::kFloat).contiguous();
  at::Tensor o = out.contiguous(), l = lse.contiguous(), g = grad_out.to(q.scalar_type()).contiguous();
  const int64_t Bw = q.size(0), N = q.size(1), T2 = (2 * window - 1) * (2 * window - 1), nw = nwin_h * nwin_w;
  TORCH_CHECK(nw > 0 && Bw % nw == 0, "num_windows must be a multiple of nwin_h * nwin_w");
  TORCH_CHECK(o.sizes() == at::IntArrayRef({Bw / nw, height, width, heads * 32}) && g.sizes() == o.sizes(),
              "out / grad_out must be [B, height, width, heads*32]");
  TORCH_CHECK(l.scalar_type() == at::kFloat && l.sizes() == at::IntArrayRef({Bw, heads, N}),
              "lse must be float32 [B*nW, heads, window^2]");
  TORCH_CHECK(table.numel() == T2 * heads, "rel_table must be [(2ws-1)^2, heads]");
  at::Tensor gqkv = at::empty_like(q);
  at::Tensor part = at::empty({Bw, heads, T2}, q.options().dtype(at::kFloat));
  vs_ok(vs_window_attn_backward_image(dcode(q), fp8 ? 1 : 0, q.data_ptr(), table.data_ptr<float>(), o.data_ptr(),
                                      l.data_ptr<float>(), g.data_ptr(), gqkv.data_ptr(), part.data_ptr<float>(),
                                      as_int(Bw, "windows"), (int)heads, (int)window, (int)shift, (int)nwin_h,
                                      (int)nwin_w, as_int(height, "height"), as_int(width, "width"), (float)scale,
                                      cur_stream(q)),
        "win_attn_bwd_img");
  return {gqkv, part};
}

// ---- a11: mask head einsum('bqc,bchw->bqhw') with channels-last pixel embedding
at::Tensor mask_head_fwd(const at::Tensor& mask_embed, const at::Tensor& pixel_nhwc, int64_t height, int64_t width) {
  on_device({&mask_embed, &pixel_nhwc});
  at::Tensor E = mask_embed.contiguous(), P = pixel_nhwc.to(E.scalar_type()).contiguous();
  TORCH_CHECK(E.dim() == 3, "mask_embed must be [B, Q, C]");
  const int64_t B = E.size(0), Q = E.size(1), C = E.size(2);
  TORCH_CHECK(P.numel() == B * height * width * C, "pixel embedding must be [B, H*W, C]");
  at::Tensor out = at::empty({B, Q, height, width}, E.options().dtype(at::kFloat));
  vs_ok(vs_mask_head_forward(dcode(E), E.data_ptr(), P.data_ptr(), out.data_ptr<float>(), as_int(B, "batch"),
                             as_int(Q, "queries"), as_int(C, "channels"), as_int(height, "height"),
                             as_int(width, "width"), cur_stream(E)),
        "mask_head_fwd");
  return out;
}

// bf16, C in {128, 256}: grad_E returned; grad_pixel [B, H*W, C] written (accumulate=False)
// or added to (accumulate=True) in place -- the decoder's 10 calls share one buffer.
// Query counts above the kernel's 128 run as chunks of 128 accumulating grad_pixel.
at::Tensor mask_head_bwd(const at::Tensor& grad_logits, const at::Tensor& mask_embed, const at::Tensor& pixel_nhwc,
                         at::Tensor& grad_pixel, bool accumulate) {
  on_device({&grad_logits, &mask_embed, &pixel_nhwc, &grad_pixel});
  at::Tensor E = mask_embed.contiguous(), P = pixel_nhwc.contiguous();
  TORCH_CHECK(E.scalar_type() == at::kBFloat16 && P.scalar_type() == at::kBFloat16, "mask_head_bwd is the bf16 path");
  const int64_t B = E.size(0), Q = E.size(1), C = E.size(2), N = P.numel() / (B * C);
  TORCH_CHECK(C == 128 || C == 256, "mask_head_bwd takes 128 or 256 channels");
  TORCH_CHECK(grad_pixel.is_contiguous() && grad_pixel.sizes() == P.sizes() &&
                  grad_pixel.scalar_type() == P.scalar_type(),
              "grad_pixel must be a contiguous tensor shaped and typed like pixel_nhwc");
  at::Tensor g = grad_logits.to(at::kFloat).contiguous();
  TORCH_CHECK(g.numel() == B * Q * N, "grad_logits must be [B, Q, H, W]");
  at::Tensor gE = at::empty_like(E);
  bool acc = accumulate;
  for (int64_t q0 = 0; q0 < Q; q0 += 128) {
    const int64_t q1 = std::min(Q, q0 + 128), nq = q1 - q0;
    const bool whole = q0 == 0 && q1 == Q;
    at::Tensor gc = whole ? g : g.view({B, Q, N}).slice(1, q0, q1).contiguous();
    at::Tensor Ec = whole ? E : E.slice(1, q0, q1).contiguous();
    at::Tensor gEc = whole ? gE : at::empty_like(Ec);
    at::Tensor ws = at::empty({vs_mask_head_backward_workspace_bytes((int)B, (int)nq, (int)C)},
                              E.options().dtype(at::kByte));
    vs_ok(vs_mask_head_backward_ex(dcode(E), gc.data_ptr<float>(), Ec.data_ptr(), P.data_ptr(), gEc.data_ptr(),
                                   grad_pixel.data_ptr(), ws.data_ptr(), (int)B, (int)nq, (int)C, (int)N, 1, (int)acc,
                                   cur_stream(E)),
          "mask_head_bwd");
    if (!whole) gE.slice(1, q0, q1).copy_(gEc);
    acc = true;
  }
  return gE;
}

// next layer's blocked-key bitmask from mask logits (HF:m2f:2049-2055, row fix 1912-1914)
at::Tensor attn_bitmask(const at::Tensor& logits, int64_t target_h, int64_t target_w) {
  on_device({&logits});
  at::Tensor lg = logits.to(at::kFloat).contiguous();
  TORCH_CHECK(lg.dim() == 4, "logits must be [B, Q, H, W]");
  const int64_t B = lg.size(0), Q = lg.size(1);
  at::Tensor words = at::empty({B, Q, (target_h * target_w + 31) / 32}, lg.options().dtype(at::kInt));
  vs_ok(vs_attn_bitmask(lg.data_ptr<float>(), (uint32_t*)words.data_ptr(), as_int(B * Q, "rows"),
                        (int)lg.size(2), (int)lg.size(3), as_int(target_h, "target_h"), as_int(target_w, "target_w"),
                        cur_stream(lg)),
        "attn_bitmask");
  return words;
}

// ---- a10: masked cross-attention core
void check_xattn(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& words,
                 int64_t heads) {
  TORCH_CHECK(q.dim() == 3 && q.size(2) == heads * 32, "q must be [B, Q, heads*32]");
  TORCH_CHECK(k.sizes() == v.sizes() && k.dim() == 3 && k.size(0) == q.size(0) && k.size(2) == q.size(2),
              "k / v must be [B, S, heads*32]");
  TORCH_CHECK(words.sizes() == at::IntArrayRef({q.size(0), q.size(1), (k.size(1) + 31) / 32}),
              "bitmask does not cover the keys");
}

std::tuple<at::Tensor, at::Tensor> masked_xattn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                    const at::Tensor& words, int64_t heads, double scale) {
  on_device({&q, &k, &v, &words});
  check_xattn(q, k, v, words, heads);
  at::Tensor qc = q.contiguous(), kc = k.to(q.scalar_type()).contiguous(), vc = v.to(q.scalar_type()).contiguous();
  at::Tensor wc = words.contiguous();
  const int B = as_int(q.size(0), "batch"), Q = as_int(q.size(1), "queries"), S = as_int(k.size(1), "keys");
  at::Tensor out = at::empty_like(qc);
  at::Tensor lse = at::empty({B, heads, Q}, qc.options().dtype(at::kFloat));
  at::Tensor ws = at::empty({vs_masked_attn_workspace_bytes(B, Q, S, (int)heads)}, qc.options().dtype(at::kByte));
  vs_ok(vs_masked_attn_forward(dcode(qc), qc.data_ptr(), kc.data_ptr(), vc.data_ptr(), (const uint32_t*)wc.data_ptr(),
                               out.data_ptr(), lse.data_ptr<float>(), ws.data_ptr(), B, Q, S, (int)heads,
                               (float)scale, cur_stream(qc)),
        "masked_xattn_fwd");
  return {out, lse};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> masked_xattn_bwd(const at::Tensor& q, const at::Tensor& k,
                                                                const at::Tensor& v, const at::Tensor& words,
                                                                const at::Tensor& out, const at::Tensor& lse,
                                                                const at::Tensor& grad_out, int64_t heads,
                                                                double scale) {
  on_device({&q, &k, &v, &words, &out, &lse, &grad_out});
  check_xattn(q, k, v, words, heads);
  at::Tensor qc = q.contiguous(), kc = k.contiguous(), vc = v.contiguous(), wc = words.contiguous();
  at::Tensor oc = out.contiguous(), lc = lse.contiguous(), g = grad_out.to(q.scalar_type()).contiguous();
  TORCH_CHECK(kc.scalar_type() == qc.scalar_type() && vc.scalar_type() == qc.scalar_type(), "q / k / v dtypes differ");
  const int B = as_int(q.size(0), "batch"), Q = as_int(q.size(1), "queries"), S = as_int(k.size(1), "keys");
  TORCH_CHECK(oc.sizes() == qc.sizes() && g.sizes() == qc.sizes(), "out / grad_out must be shaped like q");
  TORCH_CHECK(lc.scalar_type() == at::kFloat && lc.sizes() == at::IntArrayRef({(int64_t)B, heads, (int64_t)Q}),
              "lse must be float32 [B, heads, Q]");
  at::Tensor gq = at::empty_like(qc), gk = at::empty_like(kc), gv = at::empty_like(vc);
  at::Tensor ws = at::empty({vs_masked_attn_workspace_bytes(B, Q, S, (int)heads)}, qc.options().dtype(at::kByte));
  vs_ok(vs_masked_attn_backward(dcode(qc), qc.data_ptr(), kc.data_ptr(), vc.data_ptr(), (const uint32_t*)wc.data_ptr(),
                                oc.data_ptr(), lc.data_ptr<float>(), g.data_ptr(), gq.data_ptr(), gk.data_ptr(),
                                gv.data_ptr(), ws.data_ptr(), B, Q, S, (int)heads, (float)scale, cur_stream(qc)),
        "masked_xattn_bwd");
  return {gq, gk, gv};
}


// ---- a10: decoder self-attention core (words: an empty tensor = no mask, [Q, nw] shared by the
// batch, or [B, Q, nw])
long long self_attn_words(const at::Tensor& words, int B, int Q, int S) {
  if (words.numel() == 0) return -1;
  const int64_t nw = (S + 31) / 32;
  TORCH_CHECK(words.scalar_type() == at::kInt && words.is_contiguous(), "words must be contiguous int32");
  if (words.dim() == 2) {
    TORCH_CHECK(words.sizes() == at::IntArrayRef({(int64_t)Q, nw}), "words must be [Q, ceil(S/32)]");
    return 0;
  }
  TORCH_CHECK(words.sizes() == at::IntArrayRef({(int64_t)B, (int64_t)Q, nw}), "words must be [B, Q, ceil(S/32)]");
  return (long long)Q * nw;
}

void check_self_attn(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int64_t heads) {
  TORCH_CHECK(q.dim() == 3 && q.size(2) == heads * 32, "q must be [B, Q, heads*32]");
  TORCH_CHECK(k.sizes() == v.sizes() && k.dim() == 3 && k.size(0) == q.size(0) && k.size(2) == q.size(2),
              "k / v must be [B, S, heads*32]");
  TORCH_CHECK(q.scalar_type() == at::kBFloat16 && k.scalar_type() == at::kBFloat16 && v.scalar_type() == at::kBFloat16,
              "self_attn takes bf16 q / k / v");
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> self_attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                 const at::Tensor& words, int64_t heads, double scale) {
  on_device({&q, &k, &v});
  check_self_attn(q, k, v, heads);
  at::Tensor qc = q.contiguous(), kc = k.contiguous(), vc = v.contiguous();
  const int B = as_int(q.size(0), "batch"), Q = as_int(q.size(1), "queries"), S = as_int(k.size(1), "keys");
  const long long wbs = self_attn_words(words, B, Q, S);
  if (wbs >= 0) on_device({&words});
  at::Tensor out = at::empty_like(qc);
  at::Tensor out32 = at::empty(qc.sizes(), qc.options().dtype(at::kFloat));
  at::Tensor lse = at::empty({B, heads, Q}, qc.options().dtype(at::kFloat));
  vs_ok(vs_self_attn_forward(VS_BF16, qc.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                             wbs >= 0 ? (const uint32_t*)words.data_ptr() : nullptr, wbs >= 0 ? wbs : 0,
                             out.data_ptr(), out32.data_ptr<float>(), lse.data_ptr<float>(), B, Q, S, (int)heads,
                             (float)scale, cur_stream(qc)),
        "self_attn_fwd");
  return {out, out32, lse};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> self_attn_bwd(const at::Tensor& q, const at::Tensor& k,
                                                             const at::Tensor& v, const at::Tensor& words,
                                                             const at::Tensor& out, const at::Tensor& lse,
                                                             const at::Tensor& grad_out, int64_t heads, double scale) {
  on_device({&q, &k, &v, &out, &lse, &grad_out});
  check_self_attn(q, k, v, heads);
  at::Tensor qc = q.contiguous(), kc = k.contiguous(), vc = v.contiguous();
  at::Tensor oc = out.contiguous(), lc = lse.contiguous(), g = grad_out.to(at::kBFloat16).contiguous();
  const int B = as_int(q.size(0), "batch"), Q = as_int(q.size(1), "queries"), S = as_int(k.size(1), "keys");
  TORCH_CHECK(oc.sizes() == qc.sizes() && g.sizes() == qc.sizes() && oc.scalar_type() == at::kFloat,
              "out (the forward's f32 copy) / grad_out must be shaped like q");
  TORCH_CHECK(lc.scalar_type() == at::kFloat && lc.sizes() == at::IntArrayRef({(int64_t)B, heads, (int64_t)Q}),
              "lse must be float32 [B, heads, Q]");
  const long long wbs = self_attn_words(words, B, Q, S);
  if (wbs >= 0) on_device({&words});
  at::Tensor gq = at::empty_like(qc), gk = at::empty_like(kc), gv = at::empty_like(vc);
  vs_ok(vs_self_attn_backward(VS_BF16, qc.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                              wbs >= 0 ? (const uint32_t*)words.data_ptr() : nullptr, wbs >= 0 ? wbs : 0,
                              oc.data_ptr<float>(), lc.data_ptr<float>(), g.data_ptr(), gq.data_ptr(), gk.data_ptr(),
                              gv.data_ptr(), B, Q, S, (int)heads, (float)scale, cur_stream(qc)),
        "self_attn_bwd");
  return {gq, gk, gv};
}

}  // namespace

TORCH_LIBRARY(visionseg, m) {
  m.def("msda_fwd(Tensor value, Tensor spatial_shapes, Tensor level_start_index, Tensor sampling_loc, "
        "Tensor attn_weight, int im2col_step) -> Tensor");
  m.def("msda_bwd(Tensor value, Tensor spatial_shapes, Tensor level_start_index, Tensor sampling_loc, "
        "Tensor attn_weight, Tensor grad_output, int im2col_step, bool f32_grad_value=False) -> (Tensor, Tensor, Tensor)");
  m.def("swin_window_fwd(Tensor x, int window, int shift) -> Tensor");
  m.def("swin_window_bwd(Tensor windows, int batch, int height, int width, int window, int shift) -> Tensor");
  m.def("win_attn_fwd(Tensor qkv, Tensor rel_table, int heads, int window, int shift, int nwin_h, int nwin_w, "
        "float scale, bool fp8=False) -> (Tensor, Tensor)");
  m.def("win_attn_bwd(Tensor qkv, Tensor rel_table, Tensor out, Tensor lse, Tensor grad_out, int heads, int window, "
        "int shift, int nwin_h, int nwin_w, float scale, bool fp8=False, bool table_partials=False) -> (Tensor, Tensor)");
  m.def("win_attn_fwd_img(Tensor qkv, Tensor rel_table, int heads, int window, int shift, int nwin_h, int nwin_w, "
        "int height, int width, float scale, bool fp8) -> (Tensor, Tensor)");
  m.def("win_attn_bwd_img(Tensor qkv, Tensor rel_table, Tensor out, Tensor lse, Tensor grad_out, int heads, "
        "int window, int shift, int nwin_h, int nwin_w, int height, int width, float scale, bool fp8) "
        "-> (Tensor, Tensor)");
  m.def("mask_head_fwd(Tensor mask_embed, Tensor pixel_nhwc, int height, int width) -> Tensor");
  m.def("mask_head_bwd(Tensor grad_logits, Tensor mask_embed, Tensor pixel_nhwc, Tensor(a!) grad_pixel, "
        "bool accumulate) -> Tensor");
  m.def("attn_bitmask(Tensor logits, int target_h, int target_w) -> Tensor");
  m.def("masked_xattn_fwd(Tensor q, Tensor k, Tensor v, Tensor words, int heads, float scale) -> (Tensor, Tensor)");
  m.def("masked_xattn_bwd(Tensor q, Tensor k, Tensor v, Tensor words, Tensor out, Tensor lse, Tensor grad_out, "
        "int heads, float scale) -> (Tensor, Tensor, Tensor)");
  m.def("self_attn_fwd(Tensor q, Tensor k, Tensor v, Tensor words, int heads, float scale) -> (Tensor, Tensor, Tensor)");
  m.def("self_attn_bwd(Tensor q, Tensor k, Tensor v, Tensor words, Tensor out, Tensor lse, Tensor grad_out, "
        "int heads, float scale) -> (Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(visionseg, CUDA, m) {
  m.impl("msda_fwd", msda_fwd);
  m.impl("msda_bwd", msda_bwd);
  m.impl("swin_window_fwd", swin_window_fwd);
  m.impl("swin_window_bwd", swin_window_bwd);
  m.impl("win_attn_fwd", win_attn_fwd);
  m.impl("win_attn_bwd", win_attn_bwd);
  m.impl("win_attn_fwd_img", win_attn_fwd_img);
  m.impl("win_attn_bwd_img", win_attn_bwd_img);
  m.impl("mask_head_fwd", mask_head_fwd);
  m.impl("mask_head_bwd", mask_head_bwd);
  m.impl("attn_bitmask", attn_bitmask);
  m.impl("masked_xattn_fwd", masked_xattn_fwd);
  m.impl("masked_xattn_bwd", masked_xattn_bwd);
  m.impl("self_attn_fwd", self_attn_fwd);
  m.impl("self_attn_bwd", self_attn_bwd);
}
