// Python bindings of the gfx950 kernels (module jax_llama_amd._C).
//
// Thin: validate dtypes/shapes/contiguity on the host (a wrong shape must never reach a kernel),
// take raw pointers and launch on torch's current HIP stream (so hipGraph capture through
// torch.cuda.graph records these launches). Kernel code lives in csrc/kernels/*.hip.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/launchers.h"

#define MODE_RESIDUAL_ID 1
#define MODE_QKV_ID 3
#define MODE_TPRESID_ID 9
#define MODE_ARGMAX_ID 8  // common.h MODE_ARGMAX

namespace {

using torch::Tensor;

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(bool cond, const char* msg) { TORCH_CHECK(cond, "jax_llama_amd._C: ", msg); }

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "jax_llama_amd._C: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), "jax_llama_amd._C: ", name, " must be contiguous");
}

void rc(int r, const char* what) {
  TORCH_CHECK(r == 0, "jax_llama_amd._C: ", what, " failed (code ", r, ")");
}

template <typename T>
T* ptr(const Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}

const jla::bf16_t* cbf(const Tensor& t) { return reinterpret_cast<const jla::bf16_t*>(t.data_ptr()); }
jla::bf16_t* bf(const Tensor& t) { return reinterpret_cast<jla::bf16_t*>(t.data_ptr()); }

// optional bf16 mirror of an fp32 residual-stream tensor (same element count)
jla::bf16_t* mirror_ptr(const c10::optional<Tensor>& mirror, int64_t numel) {
  if (!mirror.has_value()) return nullptr;
  check_gpu(*mirror, "mirror");
  check(mirror->scalar_type() == torch::kBFloat16 && mirror->numel() == numel, "mirror must be bf16, same shape");
  return bf(*mirror);
}

void embedding(Tensor ids, Tensor table, Tensor out, c10::optional<Tensor> mirror) {
  check_gpu(ids, "ids");
  check_gpu(table, "table");
  check_gpu(out, "out");
  check(ids.scalar_type() == torch::kInt32 && table.scalar_type() == torch::kBFloat16 &&
            out.scalar_type() == torch::kFloat32,
        "embedding dtypes");
  const int M = ids.numel(), D = table.size(1), V = table.size(0);
  check(out.numel() == (int64_t)M * D, "embedding out shape");
  rc(jla::embedding(ptr<int32_t>(ids), cbf(table), ptr<float>(out), mirror_ptr(mirror, out.numel()), M, D, V,
                    stream()),
     "embedding");
}

void rms_scale(Tensor x, Tensor out, double eps) {
  check_gpu(x, "x");
  check_gpu(out, "out");
  check((x.scalar_type() == torch::kFloat32 || x.scalar_type() == torch::kBFloat16) &&
            out.scalar_type() == torch::kBFloat16,
        "rms_scale dtypes");
  const int D = x.size(-1), M = x.numel() / D;
  check(out.numel() == x.numel(), "rms_scale out shape");
  if (x.scalar_type() == torch::kBFloat16)
    rc(jla::rms_scale_bf16(cbf(x), bf(out), M, D, (float)eps, stream()), "rms_scale_bf16");
  else
    rc(jla::rms_scale(ptr<float>(x), bf(out), M, D, (float)eps, stream()), "rms_scale");
}

void rmsnorm(Tensor x, Tensor w, Tensor out, double eps) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  check_gpu(out, "out");
  check(x.scalar_type() == torch::kFloat32 && w.scalar_type() == torch::kFloat32 &&
            out.scalar_type() == torch::kFloat32,
        "rmsnorm dtypes");
  const int D = x.size(-1), M = x.numel() / D;
  check(w.numel() == D && out.numel() == x.numel(), "rmsnorm shapes");
  rc(jla::rmsnorm(ptr<float>(x), ptr<float>(w), ptr<float>(out), M, D, (float)eps, stream()), "rmsnorm");
}

// h (fp32) += p (bf16 / fp32, same element count); hb = bf16(h)
void residual_add(Tensor h, Tensor p, Tensor hb) {
  check_gpu(h, "h");
  check_gpu(p, "p");
  check_gpu(hb, "hb");
  check(h.scalar_type() == torch::kFloat32 && hb.scalar_type() == torch::kBFloat16 &&
            (p.scalar_type() == torch::kBFloat16 || p.scalar_type() == torch::kFloat32),
        "residual_add dtypes");
  check(p.numel() == h.numel() && hb.numel() == h.numel() && h.numel() % 8 == 0, "residual_add shapes");
  rc(jla::residual_add(ptr<float>(h), p.data_ptr(), p.scalar_type() == torch::kBFloat16, bf(hb), h.numel(), stream()),
     "residual_add");
}

// load every byte of t with the default cache policy (Infinity Cache warm-up of the next projection's weights)
void prefetch(Tensor t, int64_t grid) {
  check(t.is_cuda() && t.is_contiguous(), "prefetch: contiguous GPU tensor");
  static unsigned* sink = nullptr;  // allocated at the first (eager) call: never inside a graph capture
  if (!sink) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(stream(), &st);
    check(st == hipStreamCaptureStatusNone, "prefetch: first call under graph capture");
    rc((int)hipMalloc(reinterpret_cast<void**>(&sink), 64), "prefetch sink");
  }
  const int64_t nbytes = t.numel() * t.element_size() / 16 * 16;
  if (grid < 0) {  // the sequential streaming-read probe (calibration): each wave one contiguous range, -grid blocks
    rc(jla::stream_probe(t.data_ptr(), nbytes, (int)-grid, sink, stream()), "stream_probe");
    return;
  }
  rc(jla::prefetch(t.data_ptr(), nbytes, (int)grid, sink, stream()), "prefetch");
}

// y [M, N] = x [M, K] @ w [N, K]^T, all fp32 (precision='highest' lm_head)
void gemm_f32(Tensor x, Tensor w, Tensor y) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  check_gpu(y, "y");
  check(x.scalar_type() == torch::kFloat32 && w.scalar_type() == torch::kFloat32 && y.scalar_type() == torch::kFloat32,
        "gemm_f32 dtypes");
  check(x.dim() == 2 && w.dim() == 2 && y.dim() == 2 && x.size(1) == w.size(1) && y.size(0) == x.size(0) &&
            y.size(1) == w.size(0),
        "gemm_f32 shapes");
  rc(jla::gemm_f32(ptr<float>(x), ptr<float>(w), ptr<float>(y), x.size(0), w.size(0), x.size(1), stream()), "gemm_f32");
}

void check_packed(const Tensor& w, int64_t n, int64_t k) {
  check_gpu(w, "weight");
  check(w.scalar_type() == torch::kBFloat16, "weight must be bf16");
  check(w.dim() == 4 && w.size(0) == n / 16 && w.size(1) == k / 32 && w.size(2) == 64 && w.size(3) == 8,
        "weight must be fragment-packed [N/16, K/32, 64, 8]");
}

void check_linear_out(const Tensor& out, int64_t m, int64_t n, int64_t mode) {
  check_gpu(out, "out");
  const int64_t ncols = (mode == 2) ? n / 2 : n;
  check(out.numel() == m * ncols, "linear out shape");
  if (mode == 1) check(out.scalar_type() == torch::kFloat32, "residual must be fp32");
  if (mode == 2) check(out.scalar_type() == torch::kBFloat16, "swiglu out must be bf16");
  if (mode == 0)
    check(out.scalar_type() == torch::kBFloat16 || out.scalar_type() == torch::kFloat32, "out must be bf16/fp32");
}

// packed-layout activation copy (common.h pack_off): bf16, >= ceil(M/16 -> 1, 2 or 4 m-tiles) * 16 rows of `cols`
int64_t packed_rows(int64_t m) { return m <= 16 ? 16 : (m <= 32 ? 32 : 64); }
jla::bf16_t* packed_ptr(const c10::optional<Tensor>& t, int64_t m, int64_t cols, const char* what) {
  if (!t.has_value()) return nullptr;
  check_gpu(*t, what);
  check(t->scalar_type() == torch::kBFloat16 && t->numel() >= packed_rows(m) * cols && cols % 32 == 0,
        "packed activation: bf16 [padded rows, cols], cols % 32 == 0");
  return bf(*t);
}

// Decode linear dispatch (gemv.hip dispatch_nt). variant: 0 / 1 = K-split GEMV (4 waves at M <= 16), 5 / 6 = 4 / 2
// tiles per workgroup, 10 = 2 tiles with a doubled ring, 20 = 2 tiles x 8 waves, 16 = split-K GEMV, packed-x 12 / 15 /
// 18 / 21 / 22 / 26 (variant ids of removed forms are not reused: profiles/r4_variant_pruning.md).
void run_skinny(const Tensor& x, const Tensor& w, int64_t n, int64_t k, void* out, int64_t mode, double rms_eps,
                bool accumulate, bool out_f32, const jla::QKVArgs* qa, int64_t variant, const Tensor& ws,
                const Tensor& tickets, const jla::bf16_t* x_packed = nullptr) {
  const int64_t m = x.size(0);
  const bool f32 = x.scalar_type() == torch::kFloat32;
  if (variant == 0) variant = 1;
  const bool xp_variant = jla::gemv_xp_variant((int)variant);
  check(xp_variant == (x_packed != nullptr), "packed-x variants (12, 15, 18, 21, 22, 26) need x_packed, the others must not");
  check(!xp_variant || !f32, "packed-x variants read bf16 activations");
  check(!(xp_variant && mode == 2 && variant == 12), "SwiGLU packed-x variants: 15, 18, 21, 22, 26");
  check(variant == 1 || variant == 5 || variant == 6 || variant == 10 || variant == 16 || variant == 20 || xp_variant,
        "unknown decode GEMV variant");
  {
    jla::QKVArgs qs = *qa;
    if (jla::gemv_split_variant((int)variant)) {
      // split-K GEMV: partial slabs + self-resetting tickets (the shared skinny workspace, sized for both)
      check_gpu(ws, "ws");
      check_gpu(tickets, "tickets");
      check(ws.scalar_type() == torch::kFloat32 && tickets.scalar_type() == torch::kInt32, "ws/tickets dtypes");
      check((size_t)ws.numel() >= jla::gemv_split_workspace_floats(m, n) && ws.numel() < (1LL << 29) &&
                tickets.numel() >= jla::gemv_split_tickets(n) && jla::gemv_split_tickets(n) > 0,
            "split-K GEMV: workspace / tickets too small, or too many column groups");
      qs.sk_ws = ptr<float>(ws);
      qs.sk_tk = ptr<int32_t>(tickets);
      qs.sk_ws_floats = (int)ws.numel();
    }
    rc(jla::linear_skinny(x_packed ? (const void*)x_packed : x.data_ptr(), f32, w.data_ptr(), out, m, n, k, mode,
                          (float)rms_eps, accumulate, out_f32, &qs, variant, stream()),
       "linear_skinny");
  }
}

void linear_skinny(Tensor x, Tensor w, int64_t n, int64_t k, Tensor out, int64_t mode, double rms_eps,
                   bool accumulate, int64_t variant, Tensor ws, Tensor tickets, c10::optional<Tensor> mirror,
                   c10::optional<Tensor> x_packed, c10::optional<Tensor> pack_out) {
  check_gpu(x, "x");
  check_packed(w, n, k);
  check(x.dim() == 2 && x.size(1) == k, "x must be [M, K]");
  check(x.scalar_type() == torch::kFloat32 || x.scalar_type() == torch::kBFloat16, "x must be fp32/bf16");
  check(mode >= 0 && mode <= 2, "linear_skinny mode");
  const int64_t m = x.size(0);
  check(m <= SKINNY_MAX_M, "linear_skinny: M too large");
  check_linear_out(out, m, n, mode);
  jla::QKVArgs qa{};
  qa.res_bf16 = mode == 1 ? mirror_ptr(mirror, out.numel()) : nullptr;
  // packed copy of the bf16 output (the residual's mirror / the SwiGLU activation): GEMV variants only
  qa.pack = packed_ptr(pack_out, m, mode == 2 ? n / 2 : n, "pack_out");
  check(!qa.pack || (mode == 1 || mode == 2), "pack_out: residual (mirror) or SwiGLU output only");
  check(!qa.pack || (variant != 0 && variant != 7), "pack_out: GEMV variants only");
  check(!qa.pack || mode != 1 || qa.res_bf16, "pack_out of a residual needs the mirror");
  run_skinny(x, w, n, k, out.data_ptr(), mode, rms_eps, accumulate, out.scalar_type() == torch::kFloat32, &qa,
             variant, ws, tickets, packed_ptr(x_packed, m, k, "x_packed"));
}

// greedy lm_head at decode M (<= 64): GEMV with a first-max epilogue -> [M][N / 16] (value, index) partials in
// `part`, then one wave per row picks the first maximum (the fp32 logits are never written)
void linear_skinny_argmax(Tensor x, Tensor w, int64_t n, int64_t k, double rms_eps, int64_t variant, Tensor part,
                          Tensor idx, Tensor val) {
  check_gpu(x, "x");
  check_packed(w, n, k);
  check(x.dim() == 2 && x.size(1) == k && (x.scalar_type() == torch::kFloat32 || x.scalar_type() == torch::kBFloat16),
        "x must be fp32/bf16 [M, K]");
  const int64_t m = x.size(0);
  check(m <= SKINNY_MAX_M, "linear_skinny_argmax: M too large");
  check(variant == 1 || variant == 5 || variant == 6 || variant == 10 || variant == 20,
        "argmax: GEMV variants only (row-major x)");
  check_gpu(part, "part");
  check(part.scalar_type() == torch::kFloat32 && part.numel() >= m * (n / 16) * 2, "argmax partials too small");
  check_gpu(idx, "idx");
  check_gpu(val, "val");
  check(idx.scalar_type() == torch::kInt32 && val.scalar_type() == torch::kFloat32 && idx.numel() == m &&
            val.numel() == m,
        "argmax outputs");
  jla::QKVArgs qa{};
  rc(jla::linear_skinny(x.data_ptr(), x.scalar_type() == torch::kFloat32, w.data_ptr(), part.data_ptr(), m, n, k,
                        MODE_ARGMAX_ID, (float)rms_eps, 0, 1, &qa, variant, stream()),
     "linear_skinny_argmax");
  rc(jla::argmax_partials(ptr<float>(part), n / 16, m, ptr<int32_t>(idx), ptr<float>(val), stream()), "argmax_partials");
}

// the decode workspace of the split-K GEMV variants (16 / 18 / 26): partial slabs + tickets
py::tuple skinny_workspace(int64_t m, int64_t n, int64_t k, int64_t mode) {
  (void)k;
  (void)mode;
  return py::make_tuple((int64_t)jla::gemv_split_workspace_floats(m, n), (int64_t)jla::gemv_split_tickets(n));
}

// RoPE + KV-cache epilogue arguments of the fused qkv projection (validated here)
jla::QKVArgs qkv_args(int64_t m, int64_t n, const Tensor& table, const Tensor& positions, const Tensor& kc,
                      const Tensor& vc, const Tensor& slot, int64_t seq_len, int64_t h, int64_t hkv, int64_t dh,
                      const Tensor& q) {
  for (auto* t : {&table, &positions, &kc, &vc, &slot, &q}) check_gpu(*t, "linear_qkv arg");
  check(n == (h + 2 * hkv) * dh && dh % 16 == 0, "qkv width");
  check(table.scalar_type() == torch::kFloat32 && table.dim() == 3 && table.size(1) == dh / 2 && table.size(2) == 2,
        "rope table must be fp32 [L, Dh/2, 2]");
  check(positions.scalar_type() == torch::kInt32 && positions.numel() == m && slot.scalar_type() == torch::kInt32,
        "positions/slot");
  check(m % seq_len == 0, "M must be B * seq_len");
  const int64_t b = m / seq_len;
  check(kc.scalar_type() == torch::kBFloat16 && kc.dim() == 4 && kc.size(0) == b && kc.size(1) == hkv &&
            kc.size(3) == dh && vc.sizes() == kc.sizes() && vc.scalar_type() == torch::kBFloat16,
        "cache shape [B, Hkv, T, Dh]");
  check(q.scalar_type() == torch::kBFloat16 && q.numel() == m * h * dh, "q out");
  jla::QKVArgs qa;
  qa.table = reinterpret_cast<const float2*>(table.data_ptr());
  qa.table_len = table.size(0);
  qa.positions = ptr<int32_t>(positions);
  qa.kc = bf(kc);
  qa.vc = bf(vc);
  qa.slot = ptr<int32_t>(slot);
  qa.S = seq_len;
  qa.H = h;
  qa.Hkv = hkv;
  qa.Dh = dh;
  qa.T = kc.size(2);
  qa.q = bf(q);
  qa.res_bf16 = nullptr;
  qa.pack = nullptr;
  return qa;
}

// fused qkv projection + RoPE + KV-cache write (decode / small M)
void linear_qkv(Tensor x, Tensor w, int64_t n, int64_t k, double rms_eps, Tensor table, Tensor positions, Tensor kc,
                Tensor vc, Tensor slot, int64_t seq_len, int64_t h, int64_t hkv, int64_t dh, Tensor q,
                int64_t variant, Tensor ws, Tensor tickets, c10::optional<Tensor> x_packed) {
  check_gpu(x, "x");
  check_packed(w, n, k);
  check(x.dim() == 2 && x.size(1) == k, "x must be [M, K]");
  check(x.scalar_type() == torch::kFloat32 || x.scalar_type() == torch::kBFloat16, "x must be fp32/bf16");
  const int64_t m = x.size(0);
  check(m <= SKINNY_MAX_M, "linear_qkv: M too large");
  jla::QKVArgs qa = qkv_args(m, n, table, positions, kc, vc, slot, seq_len, h, hkv, dh, q);
  run_skinny(x, w, n, k, nullptr, MODE_QKV_ID, rms_eps, false, false, &qa, variant, ws, tickets,
             packed_ptr(x_packed, m, k, "x_packed"));
}


// fused small-batch qkv projection + decode attention (gemv.hip qkv_attn_kernel): q [M, H, Dh] (scratch the
// attention workgroups read), the attention output out [M, H * Dh] (+ its packed copy); splits from qkv_attn_splits
void linear_qkv_attn(Tensor x, Tensor w, int64_t n, int64_t k, double rms_eps, Tensor table, Tensor positions,
                     Tensor kc, Tensor vc, Tensor slot, int64_t h, int64_t hkv, int64_t dh, Tensor q, Tensor kv_start,
                     Tensor out, c10::optional<Tensor> out_pack, Tensor ws, Tensor tickets, Tensor sync, int64_t t_cap,
                     int64_t splits, c10::optional<Tensor> x_packed, int64_t spl, c10::optional<Tensor> sk_ws,
                     c10::optional<Tensor> sk_tk, c10::optional<Tensor> o_w, int64_t o_n, int64_t o_k,
                     c10::optional<Tensor> o_h, c10::optional<Tensor> o_hb, c10::optional<Tensor> o_hb_pack,
                     int64_t tp_state) {
  check_gpu(x, "x");
  check_packed(w, n, k);
  check(x.dim() == 2 && x.size(1) == k && x.scalar_type() == torch::kBFloat16, "linear_qkv_attn: x bf16 [M, K]");
  const int64_t m = x.size(0);
  check(m <= 32, "linear_qkv_attn: M <= 32");
  jla::QKVArgs qa = qkv_args(m, n, table, positions, kc, vc, slot, 1, h, hkv, dh, q);
  for (auto* t : {&kv_start, &out, &ws, &tickets, &sync}) check_gpu(*t, "linear_qkv_attn arg");
  check(kv_start.scalar_type() == torch::kInt32 && kv_start.numel() == m, "kv_start int32 [B]");
  check(out.scalar_type() == torch::kBFloat16 && out.numel() == m * h * dh, "out bf16 [B, H * Dh]");
  check(ws.scalar_type() == torch::kFloat32 && ws.numel() >= m * hkv * splits * (h / hkv) * (dh + 4), "ws too small");
  check(tickets.scalar_type() == torch::kInt32 && tickets.numel() >= m * hkv, "tickets int32 [pairs]");
  check(sync.scalar_type() == torch::kInt32 && (size_t)sync.numel() >= jla::qkv_attn_sync_ints(),
        "sync int32 [qkv_attn_sync_ints()]");
  check(t_cap <= kc.size(2), "t_cap <= cache length");
  const jla::bf16_t* xp = packed_ptr(x_packed, m, k, "x_packed");
  check(spl == 1 || spl == 2, "linear_qkv_attn: spl 1 or 2");
  if (spl > 1) {  // the split qkv GEMV's slabs + tickets (skinny_workspace)
    check(sk_ws.has_value() && sk_tk.has_value(), "linear_qkv_attn spl 2: sk_ws and sk_tk (skinny_workspace)");
    check_gpu(*sk_ws, "sk_ws");
    check_gpu(*sk_tk, "sk_tk");
    check(sk_ws->scalar_type() == torch::kFloat32 && sk_tk->scalar_type() == torch::kInt32 &&
              sk_tk->numel() >= n / 16,
          "linear_qkv_attn: sk_ws fp32, sk_tk int32 [N / 16]");
    qa.sk_ws = ptr<float>(*sk_ws);
    qa.sk_tk = ptr<int32_t>(*sk_tk);
    qa.sk_ws_floats = (int)sk_ws->numel();
  }
  // the fused o projection (o_w): h += out @ Wo^T with the residual epilogue (tp_state 0) or the TP exchange
  jla::QKVArgs qo{};
  float* oh = nullptr;
  int o_mode = 0;
  if (o_w.has_value()) {
    check_packed(*o_w, o_n, o_k);
    check(o_k == h * dh, "linear_qkv_attn: Wo has H * Dh input columns");
    check(o_h.has_value() && o_hb.has_value(), "linear_qkv_attn: the fused o projection needs h and hb");
    check_gpu(*o_h, "h");
    check_gpu(*o_hb, "hb");
    check(o_h->scalar_type() == torch::kFloat32 && o_h->numel() == m * o_n && o_hb->scalar_type() == torch::kBFloat16 &&
              o_hb->numel() == m * o_n, "linear_qkv_attn: h fp32 / hb bf16 [M, N_o]");
    const int og = jla::qkv_attn_o_groups((int)m, (int)(h / hkv), (int)o_n, (int)o_k);
    check(og > 0, "linear_qkv_attn: the o projection cannot be fused at this shape (qkv_attn_o_groups)");
    oh = ptr<float>(*o_h);
    qo.res_bf16 = bf(*o_hb);
    qo.pack = packed_ptr(o_hb_pack, m, o_n, "o_hb_pack");
    o_mode = MODE_RESIDUAL_ID;
    if (tp_state) {
      void* st = reinterpret_cast<void*>(tp_state);
      check(og <= jla::CAR_WG_COUNTERS && og * jla::TPRES_REGION <= jla::car_max_bytes(st),
            "linear_qkv_attn: too many o workgroups for the TP buffer");
      qo.tp = jla::car_device(st);
      o_mode = MODE_TPRESID_ID;
    }
  }
  rc(jla::linear_qkv_attn(xp ? xp : cbf(x), w.data_ptr(), m, n, k, (float)rms_eps, qa, xp != nullptr, bf(out),
                          packed_ptr(out_pack, m, h * dh, "out_pack"), ptr<int32_t>(kv_start), ptr<float>(ws),
                          ptr<int32_t>(tickets), ptr<int32_t>(sync), (int)t_cap, (int)splits, (int)spl, stream(),
                          o_w.has_value() ? o_w->data_ptr() : nullptr, oh, (int)o_n, (int)o_k, o_mode,
                          o_w.has_value() ? &qo : nullptr),
     "linear_qkv_attn");
}

void check_gemm_ws(const c10::optional<Tensor>& ws, int64_t ksplit, int64_t m, int64_t n, bool rms = false) {
  if (ksplit <= 1) return;
  check(ws.has_value(), "gemm: split-K needs a workspace");
  check_gpu(*ws, "gemm ws");
  check(ws->scalar_type() == torch::kFloat32 && ws->numel() >= ksplit * m * (n + (rms ? 1 : 0)),
        "gemm ws too small");
}

// gemm5 (tiles 11 / 12) slab workspace: [ks][M][N] (+ [ks][M] norm partials) for its effective split over 64-deep stages
void check_g5_ws(const c10::optional<Tensor>& ws, int64_t k, int64_t ksplit, int64_t m, int64_t n, bool rms) {
  check(ws.has_value(), "gemm tile 11 / 12: the slab workspace is required (any split)");
  check_gpu(*ws, "gemm ws");
  const int64_t eks = jla::gemm5_ksplit((int)k, (int)ksplit);
  check(ws->scalar_type() == torch::kFloat32 && ws->numel() >= eks * m * (n + (rms ? 1 : 0)), "gemm ws too small");
}

// Tiled MFMA GEMM; ksplit > 1 -> split-K partials in ws + fixed-order reduce/epilogue kernel.
// rms_ws: optional fp32 scratch (>= M floats) for the row statistic of the fused norm on gemm4 plans without a K
// split (computed ahead of the GEMM by rms_rowinv); absent: the statistic is summed inside the main loop.
static float* rms_ws_ptr(const c10::optional<Tensor>& rws, int64_t m, size_t* floats) {
  *floats = 0;
  if (!rws.has_value()) return nullptr;
  check_gpu(*rws, "rms_ws");
  check(rws->scalar_type() == torch::kFloat32 && rws->numel() >= m, "rms_ws: fp32, >= M floats");
  *floats = rws->numel();
  return ptr<float>(*rws);
}

void gemm(Tensor x, Tensor w, int64_t n, int64_t k, Tensor out, int64_t mode, bool accumulate,
          c10::optional<Tensor> mirror, int64_t ksplit, c10::optional<Tensor> ws, double rms_eps, int64_t tile,
          c10::optional<Tensor> pack_out, c10::optional<Tensor> rms_ws) {
  check_gpu(x, "x");
  check_packed(w, n, k);
  check(x.dim() == 2 && x.size(1) == k && x.scalar_type() == torch::kBFloat16, "x must be bf16 [M, K]");
  check(mode >= 0 && mode <= 2, "gemm mode");
  check(rms_eps < 0 || mode != 1, "gemm: fused RMS is not available in residual mode");
  const int64_t m = x.size(0);
  check_linear_out(out, m, n, mode);
  jla::bf16_t* mir = mode == 1 ? mirror_ptr(mirror, out.numel()) : nullptr;
  // packed copy of the bf16 output (decode M <= 64; the residual's mirror / the SwiGLU activation): written by the
  // split-K reduce epilogue, so only on that path
  jla::QKVArgs pqa{};
  if (pack_out.has_value()) {
    check(m <= SKINNY_MAX_M && (mode == 1 || mode == 2) && (mode != 1 || mir), "gemm pack_out: decode M, residual "
          "(with its mirror) or SwiGLU");
    check(ksplit > 1 || tile == 11 || tile == 12, "gemm pack_out: the split-K reduce-kernel path only");
    pqa.pack = packed_ptr(pack_out, m, mode == 2 ? n / 2 : n, "pack_out");
  }
  if (tile == 11 || tile == 12) {  // gemm5 (weight-streaming) partial slabs + the reduce kernel's epilogue, any split
    check_g5_ws(ws, k, ksplit, m, n, rms_eps >= 0);
    rc(jla::gemm(cbf(x), w.data_ptr(), out.data_ptr(), m, n, k, mode, accumulate,
                 out.scalar_type() == torch::kFloat32, mir, pqa.pack ? &pqa : nullptr, ptr<float>(*ws), ws->numel(),
                 ksplit, stream(), (float)rms_eps, (int)tile, nullptr, 0),
       "gemm");
    return;
  }
  check_gemm_ws(ws, ksplit, m, n, rms_eps >= 0);
  size_t rfl = 0;
  float* rws = rms_ws_ptr(rms_ws, m, &rfl);
  rc(jla::gemm(cbf(x), w.data_ptr(), out.data_ptr(), m, n, k, mode, accumulate,
               out.scalar_type() == torch::kFloat32, mir, pqa.pack ? &pqa : nullptr,
               ksplit > 1 ? ptr<float>(*ws) : nullptr, ksplit > 1 ? ws->numel() : 0, ksplit, stream(),
               (float)rms_eps, (int)tile, rws, rfl),
     "gemm");
}

// Tiled split-K qkv projection with the RoPE + KV-cache write in the reduce epilogue (x: bf16; rms_eps >= 0
// applies the fused RMSNorm statistic, otherwise x must already be scaled).
void gemm_qkv(Tensor x, Tensor w, int64_t n, int64_t k, Tensor table, Tensor positions, Tensor kc, Tensor vc,
              Tensor slot, int64_t seq_len, int64_t h, int64_t hkv, int64_t dh, Tensor q, int64_t ksplit,
              c10::optional<Tensor> ws, double rms_eps, int64_t tile, c10::optional<Tensor> rms_ws) {
  check_gpu(x, "x");
  check_packed(w, n, k);
  check(x.dim() == 2 && x.size(1) == k && x.scalar_type() == torch::kBFloat16, "x must be bf16 [M, K]");
  const int64_t m = x.size(0);
  jla::QKVArgs qa = qkv_args(m, n, table, positions, kc, vc, slot, seq_len, h, hkv, dh, q);
  if (tile == 11 || tile == 12) {  // gemm5 partial slabs, RoPE / KV write in the reduce kernel
    check_g5_ws(ws, k, ksplit, m, n, rms_eps >= 0);
    rc(jla::gemm(cbf(x), w.data_ptr(), nullptr, m, n, k, MODE_QKV_ID, 0, 0, nullptr, &qa, ptr<float>(*ws), ws->numel(),
                 ksplit, stream(), (float)rms_eps, (int)tile, nullptr, 0),
       "gemm_qkv");
    return;
  }
  if (ksplit <= 1) {  // no K split: the GEMM's own RoPE / KV-write epilogue (default FA pipeline, fused norm)
    check(rms_eps >= 0 && jla::gemm_qkv_direct_ok((int)m, (int)tile, (int)k), "gemm_qkv without a K split: 256 x 256 FA "
          "tiles with the fused norm (gemm_qkv_direct_ok)");
    size_t rfl = 0;
    float* rws = rms_ws_ptr(rms_ws, m, &rfl);
    rc(jla::gemm(cbf(x), w.data_ptr(), nullptr, m, n, k, MODE_QKV_ID, 0, 0, nullptr, &qa, nullptr, 0, 1, stream(),
                 (float)rms_eps, (int)tile, rws, rfl),
       "gemm_qkv");
    return;
  }
  check(ws.has_value(), "gemm_qkv: a K split needs the slab workspace");
  check_gemm_ws(ws, ksplit, m, n, rms_eps >= 0);
  rc(jla::gemm(cbf(x), w.data_ptr(), nullptr, m, n, k, MODE_QKV_ID, 0, 0, nullptr, &qa, ptr<float>(*ws), ws->numel(),
               ksplit, stream(), (float)rms_eps, (int)tile),
     "gemm_qkv");
}

void rope_kv_write(Tensor qkv, Tensor table, Tensor positions, Tensor kc, Tensor vc, Tensor slot, int64_t seq_len,
                   int64_t h, int64_t hkv, int64_t dh, Tensor q) {
  for (auto* t : {&qkv, &table, &positions, &kc, &vc, &slot, &q}) check_gpu(*t, "rope_kv_write arg");
  check(qkv.scalar_type() == torch::kBFloat16 && kc.scalar_type() == torch::kBFloat16 &&
            vc.scalar_type() == torch::kBFloat16 && q.scalar_type() == torch::kBFloat16,
        "rope_kv_write bf16 tensors");
  check(table.scalar_type() == torch::kFloat32 && table.dim() == 3 && table.size(1) == dh / 2 && table.size(2) == 2,
        "rope table must be fp32 [L, Dh/2, 2]");
  check(positions.scalar_type() == torch::kInt32 && slot.scalar_type() == torch::kInt32, "int32 positions/slot");
  const int64_t m = qkv.size(0);
  check(qkv.dim() == 2 && qkv.size(1) == (h + 2 * hkv) * dh, "qkv shape");
  check(positions.numel() == m && m % seq_len == 0, "positions shape");
  const int64_t b = m / seq_len;
  check(kc.dim() == 4 && kc.size(0) == b && kc.size(1) == hkv && kc.size(3) == dh && vc.sizes() == kc.sizes(),
        "cache shape [B, Hkv, T, Dh]");
  check(q.numel() == m * h * dh, "q out shape");
  rc(jla::rope_kv_write(cbf(qkv), ptr<float>(table), table.size(0), ptr<int32_t>(positions), bf(kc), bf(vc),
                        ptr<int32_t>(slot), m, seq_len, h, hkv, dh, kc.size(2), bf(q), stream()),
     "rope_kv_write");
}

void check_attn(const Tensor& q, const Tensor& kc, const Tensor& vc, const Tensor& slot, const Tensor& kv_start,
                const c10::optional<Tensor>& key_mask, const Tensor& out) {
  for (auto* t : {&q, &kc, &vc, &slot, &kv_start, &out}) check_gpu(*t, "attention arg");
  check(q.scalar_type() == torch::kBFloat16 && kc.scalar_type() == torch::kBFloat16 &&
            vc.scalar_type() == torch::kBFloat16 && out.scalar_type() == torch::kBFloat16,
        "attention bf16 tensors");
  check(q.dim() == 4 && kc.dim() == 4 && kc.sizes() == vc.sizes(), "attention shapes");
  check(kc.size(0) == q.size(0) && kc.size(3) == q.size(3), "cache/q shape mismatch");
  check(q.size(2) % kc.size(1) == 0, "H must be a multiple of Hkv");
  check(slot.scalar_type() == torch::kInt32 && kv_start.scalar_type() == torch::kInt32 &&
            kv_start.numel() == q.size(0),
        "slot/kv_start");
  check(out.numel() == q.numel(), "attention out shape");
  if (key_mask.has_value()) {
    check_gpu(*key_mask, "key_mask");
    check(key_mask->scalar_type() == torch::kUInt8 && key_mask->dim() == 2 && key_mask->size(0) == q.size(0),
          "key_mask must be uint8 [B, L]");
  }
}

void attn_decode(Tensor q, Tensor kc, Tensor vc, Tensor slot, Tensor kv_start, c10::optional<Tensor> key_mask,
                 Tensor out, Tensor ws, Tensor tickets, int64_t t_cap, int64_t nsplit, c10::optional<Tensor> out_pack) {
  check_attn(q, kc, vc, slot, kv_start, key_mask, out);
  check(q.size(1) == 1, "attn_decode: one query per row");
  const int64_t b = q.size(0), h = q.size(2), dh = q.size(3), hkv = kc.size(1), T = kc.size(2);
  check(t_cap <= T, "t_cap exceeds the cache length");
  check_gpu(ws, "ws");
  check_gpu(tickets, "tickets");
  check(ws.scalar_type() == torch::kFloat32 && ws.numel() >= b * h * nsplit * (dh + 2), "workspace too small");
  check(tickets.scalar_type() == torch::kInt32 && tickets.numel() >= b * hkv, "tickets too small");
  const uint8_t* km = key_mask.has_value() ? ptr<uint8_t>(*key_mask) : nullptr;
  const int ml = key_mask.has_value() ? key_mask->size(1) : 0;
  rc(jla::attn_decode(cbf(q), cbf(kc), cbf(vc), ptr<int32_t>(slot), ptr<int32_t>(kv_start), km, ml, bf(out),
                      ptr<float>(ws), ptr<int32_t>(tickets), b, h, hkv, dh, T, t_cap, nsplit, stream(),
                      packed_ptr(out_pack, b, h * dh, "out_pack")),
     "attn_decode");
}

void attn_prefill(Tensor q, Tensor kc, Tensor vc, Tensor slot, Tensor kv_start, c10::optional<Tensor> key_mask,
                  Tensor out) {
  check_attn(q, kc, vc, slot, kv_start, key_mask, out);
  const uint8_t* km = key_mask.has_value() ? ptr<uint8_t>(*key_mask) : nullptr;
  const int ml = key_mask.has_value() ? key_mask->size(1) : 0;
  rc(jla::attn_prefill(cbf(q), cbf(kc), cbf(vc), ptr<int32_t>(slot), ptr<int32_t>(kv_start), km, ml, bf(out),
                       q.size(0), q.size(1), q.size(2), kc.size(1), q.size(3), kc.size(2), stream()),
     "attn_prefill");
}

void argmax(Tensor logits, Tensor idx, Tensor val) {
  check_gpu(logits, "logits");
  check_gpu(idx, "idx");
  check_gpu(val, "val");
  check(logits.scalar_type() == torch::kFloat32 && logits.dim() == 2, "logits must be fp32 [B, V]");
  check(idx.scalar_type() == torch::kInt32 && val.scalar_type() == torch::kFloat32 &&
            idx.numel() == logits.size(0) && val.numel() == logits.size(0),
        "argmax outputs");
  rc(jla::argmax(ptr<float>(logits), logits.size(0), logits.size(1), ptr<int32_t>(idx), ptr<float>(val), stream()),
     "argmax");
}

// Greedy lm_head: tiled GEMM (fused RMS when rms_eps >= 0) with the argmax in its epilogue; the fp32
// logits are never written. ws: fp32 >= gemm_argmax_workspace(m, n) floats.
void gemm_argmax(Tensor x, Tensor w, int64_t n, int64_t k, Tensor ws, double rms_eps, Tensor idx, Tensor val,
                 c10::optional<Tensor> rms_ws) {
  check_gpu(x, "x");
  check_packed(w, n, k);
  check(x.dim() == 2 && x.size(1) == k && x.scalar_type() == torch::kBFloat16, "x must be bf16 [M, K]");
  const int64_t m = x.size(0);
  check_gpu(ws, "ws");
  check(ws.scalar_type() == torch::kFloat32 && (size_t)ws.numel() >= jla::gemm_argmax_workspace_floats(m, n),
        "gemm_argmax ws too small");
  check_gpu(idx, "idx");
  check_gpu(val, "val");
  check(idx.scalar_type() == torch::kInt32 && val.scalar_type() == torch::kFloat32 && idx.numel() == m &&
            val.numel() == m,
        "gemm_argmax outputs");
  size_t rfl = 0;
  float* rws = rms_ws_ptr(rms_ws, m, &rfl);
  rc(jla::gemm_argmax(cbf(x), w.data_ptr(), ptr<float>(ws), ws.numel(), m, n, k, (float)rms_eps, ptr<int32_t>(idx),
                      ptr<float>(val), stream(), rws, rfl),
     "gemm_argmax");
}

// stage 1 of the sampler: per-4096-chunk top-K candidates (global indices = local + idx_offset)
void topk_chunk(Tensor logits, int64_t k, int64_t idx_offset, Tensor cv, Tensor ci) {
  for (auto* t : {&logits, &cv, &ci}) check_gpu(*t, "topk_chunk arg");
  check(logits.scalar_type() == torch::kFloat32 && logits.dim() == 2, "logits must be fp32 [B, V]");
  const int64_t b = logits.size(0), v = logits.size(1);
  check(k >= 1 && k <= 64 && k <= v, "topk_chunk: 1 <= k <= min(64, V)");
  const int64_t c = (int64_t)jla::topk_chunks(v) * k;
  check(cv.scalar_type() == torch::kFloat32 && ci.scalar_type() == torch::kInt32 && cv.numel() == b * c &&
            ci.numel() == b * c,
        "topk_chunk: candidates must be [B, chunks*k] fp32/int32");
  rc(jla::topk_chunk(ptr<float>(logits), b, v, k, idx_offset, ptr<float>(cv), ptr<int32_t>(ci), stream()),
     "topk_chunk");
}

// stage 2: merge [B, C] candidates -> sorted top-K (mode 0) or one sampled token per row (mode 1)
void topk_merge(Tensor cv, Tensor ci, int64_t k, int64_t mode, c10::optional<Tensor> out_v,
                c10::optional<Tensor> out_i, c10::optional<Tensor> nxt, double temperature, double top_p,
                int64_t seed, c10::optional<Tensor> step) {
  check_gpu(cv, "cv");
  check_gpu(ci, "ci");
  check(cv.dim() == 2 && cv.sizes() == ci.sizes() && cv.scalar_type() == torch::kFloat32 &&
            ci.scalar_type() == torch::kInt32,
        "topk_merge: candidates [B, C] fp32/int32");
  const int64_t b = cv.size(0), c = cv.size(1);
  check(k >= 1 && k <= 64 && k <= c && c <= 4096, "topk_merge: 1 <= k <= 64, k <= C <= 4096");
  float* ov = nullptr;
  int32_t* oi = nullptr;
  int32_t* nx = nullptr;
  const int32_t* st = nullptr;
  if (mode == 0) {
    check(out_v.has_value() && out_i.has_value(), "topk_merge mode 0 needs out_v/out_i");
    check_gpu(*out_v, "out_v");
    check_gpu(*out_i, "out_i");
    check(out_v->scalar_type() == torch::kFloat32 && out_i->scalar_type() == torch::kInt32 &&
              out_v->numel() == b * k && out_i->numel() == b * k,
          "topk_merge outputs [B, k]");
    ov = ptr<float>(*out_v);
    oi = ptr<int32_t>(*out_i);
  } else {
    check(mode == 1 && nxt.has_value() && step.has_value(), "topk_merge mode 1 needs nxt and step");
    check_gpu(*nxt, "nxt");
    check_gpu(*step, "step");
    check(nxt->scalar_type() == torch::kInt32 && nxt->numel() == b && step->scalar_type() == torch::kInt32,
          "topk_merge nxt [B] / step [1] int32");
    check(temperature > 0, "topk_merge: temperature > 0");
    nx = ptr<int32_t>(*nxt);
    st = ptr<int32_t>(*step);
  }
  rc(jla::topk_merge(ptr<float>(cv), ptr<int32_t>(ci), b, c, k, mode, ov, oi, nx, (float)temperature, (float)top_p,
                     (uint64_t)seed, st, stream()),
     "topk_merge");
}

void decode_update(Tensor nxt, Tensor finished, Tensor sequences, Tensor cur_len, Tensor tokens, Tensor positions,
                   Tensor slot, int64_t pad, int64_t eos) {
  for (auto* t : {&nxt, &finished, &sequences, &cur_len, &tokens, &positions, &slot}) {
    check_gpu(*t, "decode_update arg");
    check(t->scalar_type() == torch::kInt32, "decode_update: int32 tensors");
  }
  const int64_t b = nxt.numel();
  check(finished.numel() == b && tokens.numel() == b && positions.numel() == b && sequences.dim() == 2 &&
            sequences.size(0) == b,
        "decode_update shapes");
  rc(jla::decode_update(ptr<int32_t>(nxt), ptr<int32_t>(finished), ptr<int32_t>(sequences), ptr<int32_t>(cur_len),
                        ptr<int32_t>(tokens), ptr<int32_t>(positions), ptr<int32_t>(slot), b, sequences.size(1), pad,
                        eos, stream()),
     "decode_update");
}

// ---- custom all-reduce (allreduce.hip) -------------------------------------------------------
py::tuple car_alloc(int64_t max_bytes, int64_t world) {
  void* buf = nullptr;
  void* sig = nullptr;
  hipIpcMemHandle_t hb, hs;
  rc(jla::car_alloc(max_bytes, world, &buf, &sig, &hb, &hs), "car_alloc");
  return py::make_tuple((int64_t)(uintptr_t)buf, (int64_t)(uintptr_t)sig,
                        py::bytes(reinterpret_cast<const char*>(&hb), sizeof(hb)),
                        py::bytes(reinterpret_cast<const char*>(&hs), sizeof(hs)));
}

int64_t car_init(int64_t rank, int64_t world, int64_t max_bytes, int64_t buf, int64_t sig, std::vector<std::string> hbufs,
                 std::vector<std::string> hsigs, double timeout_s) {
  check((int64_t)hbufs.size() == world && (int64_t)hsigs.size() == world, "car_init: one handle per rank");
  std::vector<hipIpcMemHandle_t> hb(world), hs(world);
  for (int64_t p = 0; p < world; ++p) {
    check(hbufs[p].size() == sizeof(hipIpcMemHandle_t) && hsigs[p].size() == sizeof(hipIpcMemHandle_t),
          "car_init: handle size");
    std::memcpy(&hb[p], hbufs[p].data(), sizeof(hipIpcMemHandle_t));
    std::memcpy(&hs[p], hsigs[p].data(), sizeof(hipIpcMemHandle_t));
  }
  void* state = nullptr;
  rc(jla::car_init(rank, world, max_bytes, reinterpret_cast<void*>(buf), reinterpret_cast<void*>(sig), hb.data(),
                   hs.data(), timeout_s, &state),
     "car_init");
  return (int64_t)(uintptr_t)state;
}

// out = sum over the TP group of in (same dtype, bf16/fp32)
void car_allreduce(int64_t state, Tensor in, Tensor out, bool two_shot) {
  check_gpu(in, "in");
  check_gpu(out, "out");
  check(in.scalar_type() == out.scalar_type() && in.numel() == out.numel(), "car_allreduce in/out");
  check(in.scalar_type() == torch::kBFloat16 || in.scalar_type() == torch::kFloat32, "car_allreduce dtype");
  const int64_t nbytes = in.numel() * in.element_size();
  check(nbytes % 16 == 0, "car_allreduce: bytes % 16");
  rc(jla::car_reduce(reinterpret_cast<void*>(state), 0, in.data_ptr(), out.data_ptr(), nullptr, nullptr, nbytes,
                     in.scalar_type() == torch::kBFloat16, two_shot, stream()),
     "car_allreduce");
}

// residual all-reduce of a row-parallel projection: h (fp32) += sum over ranks of partial; hb = bf16(h)
void car_allreduce_residual(int64_t state, Tensor partial, Tensor h, Tensor hb, bool two_shot,
                            c10::optional<Tensor> hb_pack) {
  check_gpu(partial, "partial");
  check_gpu(h, "h");
  check_gpu(hb, "hb");
  check(partial.scalar_type() == torch::kBFloat16 || partial.scalar_type() == torch::kFloat32, "partial dtype");
  check(h.scalar_type() == torch::kFloat32 && hb.scalar_type() == torch::kBFloat16, "h fp32 / hb bf16");
  check(h.numel() == partial.numel() && hb.numel() == partial.numel(), "residual shapes");
  const int64_t nbytes = partial.numel() * partial.element_size();
  check(nbytes % 16 == 0, "car_allreduce_residual: bytes % 16");
  const int64_t cols = h.size(-1);
  jla::bf16_t* hp = packed_ptr(hb_pack, h.numel() / cols, cols, "hb_pack");
  rc(jla::car_reduce(reinterpret_cast<void*>(state), 1, partial.data_ptr(), nullptr, ptr<float>(h), bf(hb), nbytes,
                     partial.scalar_type() == torch::kBFloat16, two_shot, stream(), hp, hp ? (int)cols : 0),
     "car_allreduce_residual");
}

// fused row-parallel decode projection (gemv.hip MODE_TPRESID): h (fp32) += sum over the TP group of x @ W^T, the
// partials exchanged as tagged granules in the GEMV's own epilogue; hb = bf16(h) (+ its packed copy). `state` is a
// custom all-reduce instance reserved for this path (its per-workgroup counters must not be shared)
void linear_tp_residual(int64_t state, Tensor x, Tensor w, int64_t n, int64_t k, Tensor h, Tensor hb, int64_t variant,
                        c10::optional<Tensor> x_packed, c10::optional<Tensor> hb_pack, c10::optional<Tensor> ws,
                        c10::optional<Tensor> tickets) {
  check_gpu(x, "x");
  check_gpu(h, "h");
  check_gpu(hb, "hb");
  check_packed(w, n, k);
  check(x.dim() == 2 && x.size(1) == k && x.scalar_type() == torch::kBFloat16, "x must be bf16 [M, K]");
  const int64_t m = x.size(0);
  check(m >= 1 && m <= SKINNY_MAX_M, "linear_tp_residual: 1 <= M <= 64");
  check(h.scalar_type() == torch::kFloat32 && h.numel() == m * n && hb.scalar_type() == torch::kBFloat16 &&
            hb.numel() == m * n, "h fp32 / hb bf16 [M, N]");
  check(variant != 0 && variant != 4 && variant != 7, "linear_tp_residual: GEMV variants only");
  void* st = reinterpret_cast<void*>(state);
  // one TPRES_REGION per workgroup (at most 4096 workgroups: the counters), inside one slot
  const int64_t groups = n / 16;  // upper bound (1 tile per workgroup)
  check(groups <= jla::CAR_WG_COUNTERS && groups * jla::TPRES_REGION <= jla::car_max_bytes(st),
        "linear_tp_residual: too many workgroups for the buffer");
  jla::QKVArgs qa{};
  qa.res_bf16 = bf(hb);
  qa.pack = packed_ptr(hb_pack, m, n, "hb_pack");
  qa.tp = jla::car_device(st);
  // split-K variants (16 / 18 / 26) take the shared decode workspace: only the last arriver of a column group exchanges
  run_skinny(x, w, n, k, h.data_ptr(), MODE_TPRESID_ID, -1.0, true, true, &qa, variant, ws ? *ws : Tensor(),
             tickets ? *tickets : Tensor(), packed_ptr(x_packed, m, k, "x_packed"));
}

// Row-parallel tiled projection (decode batches past the GEMV's rows) with the TP all-reduce and residual add in its
// split-K reduce (gemm.hip gemm_reduce_tp_kernel): h (fp32) += sum over the group of x @ W^T, hb = bf16(h). A split plan
// (ksplit > 1, or gemm5 tiles 11 / 12) and the shared gemm workspace; one exchange region per 4096 output elements.
void gemm_tp_residual(int64_t state, Tensor x, Tensor w, int64_t n, int64_t k, Tensor h, Tensor hb, int64_t ksplit,
                      Tensor ws, int64_t tile) {
  check_gpu(x, "x");
  check_gpu(h, "h");
  check_gpu(hb, "hb");
  check_packed(w, n, k);
  check(x.dim() == 2 && x.size(1) == k && x.scalar_type() == torch::kBFloat16, "x must be bf16 [M, K]");
  const int64_t m = x.size(0);
  check(h.scalar_type() == torch::kFloat32 && h.numel() == m * n && hb.scalar_type() == torch::kBFloat16 &&
            hb.numel() == m * n, "h fp32 / hb bf16 [M, N]");
  void* st = reinterpret_cast<void*>(state);
  const int64_t groups = jla::gemm_tp_groups((int)m, (int)n);
  check(groups <= jla::CAR_WG_COUNTERS && groups * jla::TPRES_REGION <= jla::car_max_bytes(st),
        "gemm_tp_residual: the output does not fit the fused exchange buffer");
  const bool g5 = tile == 11 || tile == 12;
  check(g5 || ksplit > 1, "gemm_tp_residual: a split-K plan (the exchange lives in the reduce)");
  if (g5)
    check_g5_ws(ws, k, ksplit, m, n, false);
  else
    check_gemm_ws(ws, ksplit, m, n);
  jla::QKVArgs qa{};
  qa.tp = jla::car_device(st);
  rc(jla::gemm(cbf(x), w.data_ptr(), h.data_ptr(), m, n, k, MODE_TPRESID_ID, 1, 1, bf(hb), &qa, ptr<float>(ws),
               ws.numel(), ksplit, stream(), -1.f, (int)tile, nullptr, 0),
     "gemm_tp_residual");
}

// (value fp32, index int32) all-gathers of the vocab-parallel sampler. mode 0: out_i[n] = index of the first max over
// ranks (out_v optional); mode 1: out_v/out_i [n / k, world * k]
void car_pairs(int64_t state, int64_t mode, Tensor vals, Tensor idx, int64_t idx_offset, int64_t k,
               c10::optional<Tensor> out_v, Tensor out_i) {
  check_gpu(vals, "vals");
  check_gpu(idx, "idx");
  check_gpu(out_i, "out_i");
  check(vals.scalar_type() == torch::kFloat32 && idx.scalar_type() == torch::kInt32 &&
            out_i.scalar_type() == torch::kInt32 && vals.numel() == idx.numel(),
        "car_pairs dtypes");
  const int64_t n = vals.numel();
  auto* st = reinterpret_cast<void*>(state);
  float* ov = nullptr;
  if (out_v.has_value()) {
    check_gpu(*out_v, "out_v");
    check(out_v->scalar_type() == torch::kFloat32 && out_v->numel() == out_i.numel(), "out_v");
    ov = ptr<float>(*out_v);
  }
  if (mode == 0) {
    check(out_i.numel() == n, "car_pairs argmax out shape");
  } else {
    check(mode == 1 && ov && k > 0 && n % k == 0 && out_i.numel() == n * jla::car_world(st), "car_pairs top-k shapes");
  }
  rc(jla::car_pairs(st, (int)mode, ptr<float>(vals), ptr<int32_t>(idx), (int)idx_offset, n, (int)k, ov,
                    ptr<int32_t>(out_i), stream()),
     "car_pairs");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {  // _C, or _C_dbg for the bounds-checked build
  m.doc() = "jax_llama_amd gfx950 (MI355X) HIP kernels";
  m.attr("SKINNY_MAX_M") = SKINNY_MAX_M;
  m.attr("ARCH") = "gfx950";
  m.def("embedding", &embedding, py::arg("ids"), py::arg("table"), py::arg("out"),
        py::arg("mirror") = py::none());
  m.def("rms_scale", &rms_scale);
  m.def("rmsnorm", &rmsnorm);
  m.def("residual_add", &residual_add);
  m.def("gemm_f32", &gemm_f32);
  m.def("prefetch", &prefetch, py::arg("t"), py::arg("grid") = 128);
  m.def("linear_skinny", &linear_skinny, py::arg("x"), py::arg("w"), py::arg("n"), py::arg("k"), py::arg("out"),
        py::arg("mode"), py::arg("rms_eps"), py::arg("accumulate"), py::arg("variant"), py::arg("ws"),
        py::arg("tickets"), py::arg("mirror") = py::none(), py::arg("x_packed") = py::none(),
        py::arg("pack_out") = py::none());
  m.def("gemm", &gemm, py::arg("x"), py::arg("w"), py::arg("n"), py::arg("k"), py::arg("out"), py::arg("mode"),
        py::arg("accumulate"), py::arg("mirror") = py::none(), py::arg("ksplit") = 1, py::arg("ws") = py::none(),
        py::arg("rms_eps") = -1.0, py::arg("tile") = 0, py::arg("pack_out") = py::none(),
        py::arg("rms_ws") = py::none());
  m.def("gemm_qkv_direct_ok", [](int64_t m, int64_t tile, int64_t k) {
    return jla::gemm_qkv_direct_ok((int)m, (int)tile, (int)k) != 0;
  });
  m.def("gemm_set_g4_default", [](int64_t on) { jla::gemm_set_g4_default((int)on); });
  m.def("gemm_set_g4_group", [](int64_t gm) { jla::gemm_set_g4_group((int)gm); });
  m.def("gemm_qkv", &gemm_qkv, py::arg("x"), py::arg("w"), py::arg("n"), py::arg("k"), py::arg("table"),
        py::arg("positions"), py::arg("kc"), py::arg("vc"), py::arg("slot"), py::arg("seq_len"), py::arg("h"),
        py::arg("hkv"), py::arg("dh"), py::arg("q"), py::arg("ksplit"), py::arg("ws"), py::arg("rms_eps") = -1.0,
        py::arg("tile") = 0, py::arg("rms_ws") = py::none());
  m.def("gemm_argmax", &gemm_argmax, py::arg("x"), py::arg("w"), py::arg("n"), py::arg("k"), py::arg("ws"),
        py::arg("rms_eps"), py::arg("idx"), py::arg("val"), py::arg("rms_ws") = py::none());
  m.def("gemm_argmax_workspace", [](int64_t m, int64_t n) { return (int64_t)jla::gemm_argmax_workspace_floats(m, n); });
  m.def("gemm_ksplit", [](int64_t m, int64_t n, int64_t k) { return jla::gemm_ksplit(m, n, k); });
  m.def("rope_kv_write", &rope_kv_write);
  m.def("attn_set_impl", [](int64_t impl, int64_t waves_target) { jla::attn_set_impl(impl, waves_target); },
        py::arg("impl"), py::arg("waves_target") = 0);
  m.def("attn_decode_splits",
        [](int64_t b, int64_t hkv, int64_t t, int64_t rep) { return jla::attn_decode_splits(b, hkv, t, rep); });
  m.def("linear_qkv", &linear_qkv, py::arg("x"), py::arg("w"), py::arg("n"), py::arg("k"), py::arg("rms_eps"),
        py::arg("table"), py::arg("positions"), py::arg("kc"), py::arg("vc"), py::arg("slot"), py::arg("seq_len"),
        py::arg("h"), py::arg("hkv"), py::arg("dh"), py::arg("q"), py::arg("variant"), py::arg("ws"), py::arg("tickets"),
        py::arg("x_packed") = py::none());
  m.def("linear_qkv_attn", &linear_qkv_attn, py::arg("x"), py::arg("w"), py::arg("n"), py::arg("k"),
        py::arg("rms_eps"), py::arg("table"), py::arg("positions"), py::arg("kc"), py::arg("vc"), py::arg("slot"),
        py::arg("h"), py::arg("hkv"), py::arg("dh"), py::arg("q"), py::arg("kv_start"), py::arg("out"),
        py::arg("out_pack"), py::arg("ws"), py::arg("tickets"), py::arg("sync"), py::arg("t_cap"), py::arg("splits"),
        py::arg("x_packed") = py::none(), py::arg("spl") = 1, py::arg("sk_ws") = py::none(),
        py::arg("sk_tk") = py::none(), py::arg("o_w") = py::none(), py::arg("o_n") = 0, py::arg("o_k") = 0,
        py::arg("o_h") = py::none(), py::arg("o_hb") = py::none(), py::arg("o_hb_pack") = py::none(),
        py::arg("tp_state") = 0);
  m.def("qkv_attn_splits", [](int64_t m, int64_t b, int64_t hkv, int64_t rep, int64_t t_cap, int64_t n, int64_t cus,
                              int64_t spl, int64_t o_groups) {
    return jla::qkv_attn_splits((int)m, (int)b, (int)hkv, (int)rep, (int)t_cap, (int)n, (int)cus, (int)spl,
                                (int)o_groups);
  }, py::arg("m"), py::arg("b"), py::arg("hkv"), py::arg("rep"), py::arg("t_cap"), py::arg("n"), py::arg("cus"),
     py::arg("spl") = 1, py::arg("o_groups") = 0);
  m.def("qkv_attn_o_groups", [](int64_t m, int64_t rep, int64_t n, int64_t k) {
    return jla::qkv_attn_o_groups((int)m, (int)rep, (int)n, (int)k);
  });
  m.def("qkv_attn_sync_ints", []() { return (int64_t)jla::qkv_attn_sync_ints(); });
  m.def("qkv_attn_set_o_nt", [](int64_t nt) { jla::qkv_attn_set_o_nt((int)nt); });
  m.def("qkv_attn_set_diag", [](int64_t d) { jla::qkv_attn_set_diag((int)d); });
  m.def("qkv_attn_set_stamps", [](c10::optional<Tensor> t) {  // int64 [>= grid * 8]; None: off (keep t alive)
    if (t.has_value()) {
      check_gpu(*t, "stamps");
      check(t->scalar_type() == torch::kInt64, "stamps int64");
    }
    jla::qkv_attn_set_stamps(t.has_value() ? reinterpret_cast<unsigned long long*>(t->data_ptr()) : nullptr);
  });
  m.def("qkv_attn_occupancy", [](int64_t m, int64_t rep, int64_t spl, int64_t o_groups) {
    return jla::qkv_attn_occupancy((int)m, (int)rep, (int)spl, (int)o_groups);
  }, py::arg("m"), py::arg("rep"), py::arg("spl") = 1, py::arg("o_groups") = 0);
  m.def("attn_decode_packs", &jla::attn_decode_packs);
  m.def("skinny_workspace", &skinny_workspace);
  m.def("linear_skinny_argmax", &linear_skinny_argmax);
  m.def("gemm_tp_residual", &gemm_tp_residual, py::arg("state"), py::arg("x"), py::arg("w"), py::arg("n"), py::arg("k"),
        py::arg("h"), py::arg("hb"), py::arg("ksplit"), py::arg("ws"), py::arg("tile"));
  m.def("gemm_tp_groups", [](int64_t m, int64_t n) { return (int64_t)jla::gemm_tp_groups((int)m, (int)n); });
  m.def("linear_tp_residual", &linear_tp_residual, py::arg("state"), py::arg("x"), py::arg("w"), py::arg("n"),
        py::arg("k"), py::arg("h"), py::arg("hb"), py::arg("variant"), py::arg("x_packed") = py::none(),
        py::arg("hb_pack") = py::none(), py::arg("ws") = py::none(), py::arg("tickets") = py::none());
  m.def("bounds_error", [](bool reset) {
    const int r = reset ? 1 : 0;
    return (int64_t)(jla::jla_bounds_norm_embed(r) | jla::jla_bounds_rope_kv(r) | jla::jla_bounds_sample(r) |
                     jla::jla_bounds_gemm(r) | jla::jla_bounds_gemv(r) |
                     jla::jla_bounds_attn_decode(r) | jla::jla_bounds_attn_prefill(r));
  }, "OR of the bounds-checked debug build's error words (JLA_BOUNDS_* bits); always 0 in a release build",
        py::arg("reset") = false);
#ifdef JLA_DEBUG_BOUNDS
  m.attr("DEBUG_BOUNDS") = true;
#else
  m.attr("DEBUG_BOUNDS") = false;
#endif
  m.def("attn_set_diag", [](int64_t d) { jla::attn_set_diag((int)d); });
  // CU placement (placement.hip): streams restricted to a CU set (returned as the raw hipStream_t, wrapped by
  // torch.cuda.ExternalStream) and a census kernel recording each workgroup's HW_ID / XCC_ID
  m.def("cu_mask_stream", [](std::vector<int64_t> words) {
    std::vector<uint32_t> mk(words.begin(), words.end());
    hipStream_t s = nullptr;
    rc(jla::cu_mask_stream_create(mk.data(), (int)mk.size(), &s), "cu_mask_stream");
    return reinterpret_cast<int64_t>(s);
  });
  m.def("cu_mask_of", [](int64_t s, int64_t words) {
    std::vector<uint32_t> mk((size_t)words, 0u);
    rc(jla::cu_mask_stream_get(reinterpret_cast<hipStream_t>(s), mk.data(), (int)words), "cu_mask_of");
    return std::vector<int64_t>(mk.begin(), mk.end());
  });
  m.def("graph_kernel_nodes", [](int64_t g) {
    const int n = jla::graph_kernel_nodes(reinterpret_cast<hipGraph_t>(g));
    check(n >= 0, "graph_kernel_nodes: hipGraphGetNodes failed");
    return n;
  });
  m.def("stream_destroy", [](int64_t s) { rc(jla::stream_destroy(reinterpret_cast<hipStream_t>(s)), "stream_destroy"); });
  m.def("cu_census", [](Tensor out) {
    check_gpu(out, "out");
    check(out.scalar_type() == torch::kInt32 && out.numel() % 2 == 0, "cu_census: int32 [2 * blocks]");
    rc(jla::cu_census(reinterpret_cast<uint32_t*>(out.data_ptr()), (int)(out.numel() / 2), stream()), "cu_census");
  });
  m.def("attn_set_v3_kpg", [](int64_t m) { jla::attn_set_v3_kpg((int)m); });
  m.def("attn_set_v3_max_pairs", [](int64_t n) { jla::attn_set_v3_max_pairs((int)n); });
  m.def("attn_set_v5_max_pairs", [](int64_t n) { jla::attn_set_v5_max_pairs((int)n); });
  m.def("attn_set_v5_fold", [](int64_t n) { jla::attn_set_v5_fold((int)n); });
  m.def("clock_probe", [](int64_t iters, int64_t grid, Tensor out) {
    check(out.is_cuda() && out.scalar_type() == torch::kInt64 && out.numel() >= 3, "clock_probe: int64[3] on the GPU");
    rc(jla::clock_probe((int)iters, (int)grid, reinterpret_cast<unsigned long long*>(out.data_ptr()), stream()),
       "clock_probe");
  });
  m.def("gemm5_set_diag", [](int64_t d) { jla::gemm5_set_diag((int)d); });
  m.def("gemm5_ksplit", [](int64_t k, int64_t ks) { return jla::gemm5_ksplit((int)k, (int)ks); });
  m.def("attn_set_v6", [](int64_t mode) { jla::attn_set_v6((int)mode); });
  m.def("attn_set_v6_wpp", [](int64_t wpp) { jla::attn_set_v6_wpp((int)wpp); });
  m.def("attn_set_v6_diag", [](int64_t d) { jla::attn_set_v6_diag((int)d); });
  m.def("attn_v6_wpp", [](int64_t pairs) { return jla::attn_v6_wpp((int)pairs); });
  m.def("attn_decode", &attn_decode, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("slot"),
        py::arg("kv_start"), py::arg("key_mask").none(true), py::arg("out"), py::arg("ws"), py::arg("tickets"), py::arg("t_cap"),
        py::arg("nsplit"), py::arg("out_pack") = py::none());
  m.def("attn_prefill", &attn_prefill, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("slot"),
        py::arg("kv_start"), py::arg("key_mask").none(true), py::arg("out"));
  m.def("attn_prefill_set_impl", [](int64_t impl) { jla::attn_prefill_set_impl((int)impl); });
  m.def("argmax", &argmax);
  m.def("topk_chunks", [](int64_t v) { return jla::topk_chunks(v); });
  m.def("car_alloc", &car_alloc);
  m.def("car_init", &car_init);
  m.def("car_allreduce", &car_allreduce, py::arg("state"), py::arg("inp"), py::arg("out"), py::arg("two_shot") = false);
  m.def("car_allreduce_residual", &car_allreduce_residual, py::arg("state"), py::arg("partial"), py::arg("h"),
        py::arg("hb"), py::arg("two_shot") = false, py::arg("hb_pack") = py::none());
  m.def("car_pairs", &car_pairs, py::arg("state"), py::arg("mode"), py::arg("vals"), py::arg("idx"),
        py::arg("idx_offset"), py::arg("k"), py::arg("out_v").none(true), py::arg("out_i"));
  m.def("car_set_gran_max", [](int64_t n) { jla::car_set_gran_max(n); });
  m.def("car_set_grid", [](int64_t st, int64_t grid) {
    rc(jla::car_set_grid(reinterpret_cast<void*>(st), (int)grid), "car_set_grid");
  });
  m.def("car_error", [](int64_t st) { return jla::car_error(reinterpret_cast<void*>(st)); });
  m.def("car_destroy", [](int64_t st) { jla::car_destroy(reinterpret_cast<void*>(st)); });
  m.def("car_free", [](int64_t buf, int64_t sig) {
    jla::car_free(reinterpret_cast<void*>(buf), reinterpret_cast<void*>(sig));
  }, "free car_alloc's buffers (a failed rendezvous)");
  m.def("topk_chunk", &topk_chunk);
  m.def("topk_merge", &topk_merge, py::arg("cv"), py::arg("ci"), py::arg("k"), py::arg("mode"),
        py::arg("out_v") = py::none(), py::arg("out_i") = py::none(), py::arg("nxt") = py::none(),
        py::arg("temperature") = 1.0, py::arg("top_p") = 1.0, py::arg("seed") = 0, py::arg("step") = py::none());
  m.def("decode_update", &decode_update);
}
