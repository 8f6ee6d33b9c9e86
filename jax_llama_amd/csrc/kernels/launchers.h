// Host launchers of the gfx950 kernels (pure HIP translation units; no torch headers).
// Every launcher returns 0 on success, <0 on a shape/argument error, >0 for a hipError_t.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SKINNY_MAX_M 64

namespace jla {
typedef uint16_t bf16_t;

int embedding(const int32_t* ids, const bf16_t* table, float* out, bf16_t* mirror, int M, int D, int V,
              hipStream_t s);
int rms_scale(const float* x, bf16_t* out, int M, int D, float eps, hipStream_t s);
int rms_scale_bf16(const bf16_t* x, bf16_t* out, int M, int D, float eps, hipStream_t s);
int rms_rowinv(const bf16_t* x, float* inv, int M, int D, float eps, hipStream_t s);  // inv[M] = 1/sqrt(mean(x^2)+eps)
int residual_add(float* h, const void* p, int p_bf16, bf16_t* hb, long long n, hipStream_t s);
int prefetch(const void* p, long long nbytes, int grid, unsigned* sink, hipStream_t s);
int stream_probe(const void* p, long long nbytes, int grid, unsigned* sink, hipStream_t s);  // bytes read: per-wave contiguous ranges
int gemm_f32(const float* x, const float* w, float* y, int M, int N, int K, hipStream_t s);
int rmsnorm(const float* x, const float* w, float* out, int M, int D, float eps, hipStream_t s);

// Epilogue arguments of the fused qkv projection (MODE_QKV): RoPE + KV-cache write.
struct QKVArgs {
  const float2* table;        // [table_len, Dh/2] (cos, sin)
  int table_len;
  const int32_t* positions;   // [M]
  bf16_t* kc;                 // [B, Hkv, T, Dh] (this layer)
  bf16_t* vc;
  const int32_t* slot;        // device int32[1]: cache slot of sequence position 0
  int S, H, Hkv, Dh, T;       // tokens per sequence in this call, heads, kv heads, head dim, cache len
  bf16_t* q;                  // [M, H, Dh] rotated queries
  bf16_t* res_bf16;           // MODE_RESIDUAL: optional bf16 mirror of the updated residual (next A operand)
  bf16_t* pack;               // optional packed-layout copy (common.h pack_off) of the bf16 output: RESIDUAL -> the
                              // mirror, SWIGLU -> the activation (GEMV only; the next projection's packed-x input)
  const void* tp;             // MODE_TPRESID: the TP group's CarDevice (car.h) the partials are all-reduced through
  float* sk_ws;               // split-K GEMV variants (gemv.hip, 16 / 18 / 26): per-(group, split) partial slabs
  int32_t* sk_tk;             //   and per-group tickets (zero-initialised once, reset by each group's last arriver)
  int sk_ws_floats;           //   slab buffer size (buffer-descriptor range)
};
// MODE_TPRESID: granule bytes each workgroup of the fused row-parallel GEMV owns in every (parity, source rank) slot
constexpr int CAR_WG_COUNTERS = 4096;  // per-workgroup call counters of the fused GEMV (workgroups per launch)
constexpr long long TPRES_REGION = 64 * 64 * 4;  // up to 64 rows x 64 columns x 2 bf16 per 8-byte granule

// fused small-batch qkv projection + decode attention (gemv.hip qkv_attn_kernel): one launch; splits from
// qkv_attn_splits (0 = not applicable: run the two kernels); ws >= pairs * splits * rep * 132 floats, tickets >= pairs,
// sync >= qkv_attn_sync_ints() int32 (zeroed once, self-resetting). With o_w, the same launch also runs the o projection into the residual
// (o_mode MODE_RESIDUAL: h += out @ Wo^T + qo->res_bf16 / qo->pack mirrors; MODE_TPRESID: the TP granule exchange of
// qo->tp first); o_groups = qkv_attn_o_groups(...) (0: the o projection cannot be fused at this shape).
int qkv_attn_o_groups(int M, int rep, int N, int K);
size_t qkv_attn_sync_ints();
void qkv_attn_set_o_nt(int nt);  // o tiles per fused-o workgroup (1 / 2; tools, A/B)
int qkv_attn_splits(int M, int B, int Hkv, int rep, int t_cap, int N, int cus, int spl = 1, int o_groups = 0);
int qkv_attn_occupancy(int M, int rep, int spl = 1, int o_groups = 0);  // resident workgroups per CU it counts on
void qkv_attn_set_stamps(unsigned long long* p);  // tools: [grid][8] phase timestamps per workgroup (nullptr: off)
void qkv_attn_set_diag(int d);  // tests only: 1 = the qkv workgroups never publish (forces the timeout path)
int linear_qkv_attn(const bf16_t* x, const void* W, int M, int N, int K, float rms_eps, const QKVArgs& qa, bool xp,
                    bf16_t* out, bf16_t* out_pack, const int32_t* kv_start, float* ws, int32_t* tickets, int32_t* sync,
                    int t_cap, int splits, int spl, hipStream_t s,  // spl 2: K of the qkv GEMV over 2 (qa.sk_ws/sk_tk)
                    const void* o_w = nullptr, float* o_h = nullptr, int o_n = 0, int o_k = 0, int o_mode = 0,
                    const QKVArgs* qo = nullptr);
int linear_skinny(const void* x, int x_is_f32, const void* W, void* out, int M, int N, int K, int mode,
                  float rms_eps, int accumulate, int out_f32, const QKVArgs* qkv, int variant, hipStream_t s);
// split-K GEMV variants 16 / 18 / 26 (K over gridDim.y workgroups per column group, last arriver sums + epilogue): their slab
// floats / tickets (0 when N has too many column groups for them)
constexpr int GEMV_SPLIT_MAX_GROUPS = 1024;
size_t gemv_split_workspace_floats(int M, int N);
int gemv_split_tickets(int N);
inline bool gemv_split_variant(int v) { return v == 16 || v == 18 || v == 26; }
inline bool gemv_xp_variant(int v) { return v == 12 || v == 15 || v == 18 || v == 21 || v == 22 || v == 26; }
// 128x128-tile MFMA GEMM (gemm.hip). ksplit > 1 splits K over gridDim.z into fp32 partials
// (ws >= gemm_workspace_floats) reduced in fixed order by an epilogue kernel; MODE_QKV needs ksplit > 1.
int gemm_ksplit(int M, int N, int K);
int gemm_qkv_direct_ok(int M, int tile, int K);  // qkv without a K split: the direct RoPE / KV-write GEMM epilogue applies
// gemm4 (the 4-wave 256 x 256 kernel, tile config 7) as the tile-0 default for M > 128, K % 64 == 0 (on by default)
void gemm_set_g4_default(int on);
void gemm_set_g4_group(int gm);
int gemm5_ksplit(int K, int ksplit);
int clock_probe(int iters, int grid, unsigned long long* out, hipStream_t s);  // [cycles, 100 MHz ticks]
void gemm5_set_diag(int d);  // tools only: gemm5 ablations (wrong results)  // gemm5 (tiles 11 / 12): the effective split over 64-deep K-stages
size_t gemm_workspace_floats(int M, int N, int K);
// rms_eps >= 0: x is the UNscaled activation and each output row is scaled by rsqrt(mean(x^2) + eps)
// (fused RMSNorm; not for MODE_RESIDUAL); split-K then needs ws >= ksplit * M * (N + 1) floats.
// tile: gemm2 tile config 1 = 256x256, 2 = 128x256, 3 = 128x128, 0 = by M; 7 / 10 gemm4 (256 x 256 / 256 x 128),
// 8 gemm4 exchange split (above), 11 / 12 gemm5
// workgroups (= fused-exchange regions and call counters) of gemm()'s MODE_TPRESID reduce at M x N: the row-parallel
// projection's split-K reduce with the TP all-reduce and residual add in its epilogue (out = h, mirror = hb,
// qkv->tp = the group's CarDevice; split plans only)
int gemm_tp_groups(int M, int N);
int gemm(const bf16_t* x, const void* W, void* out, int M, int N, int K, int mode, int accumulate, int out_f32,
         bf16_t* mirror, const QKVArgs* qkv, float* ws, size_t ws_floats, int ksplit, hipStream_t s,
         float rms_eps = -1.f, int tile = 0, float* rms_ws = nullptr, size_t rms_ws_floats = 0);
// rms_ws (>= M floats): with the fused norm, a gemm4 plan without a K split computes the row statistic ahead of
// the GEMM into it (rms_rowinv) instead of inside its main loop; null: in-loop statistic
// greedy lm_head: GEMM + first-max argmax epilogue (ws >= gemm_argmax_workspace_floats(M, N) floats)
int gemm_argmax(const bf16_t* x, const void* W, float* ws, size_t ws_floats, int M, int N, int K, float rms_eps,
                int32_t* idx, float* val, hipStream_t s, float* rms_ws = nullptr, size_t rms_ws_floats = 0);
size_t gemm_argmax_workspace_floats(int M, int N);
// first max per row over [M][P] (value, index) float2 partials
int argmax_partials(const float* part, int P, int M, int32_t* idx, float* val, hipStream_t s);

int rope_kv_write(const bf16_t* qkv, const float* table, int table_len, const int32_t* positions, bf16_t* kc,
                  bf16_t* vc, const int32_t* slot, int M, int S, int H, int Hkv, int Dh, int T, bf16_t* q_out,
                  hipStream_t s);

int attn_decode_chunk(int B, int Hkv, int T, int rep);
void attn_set_v5_max_pairs(int n);
void attn_set_v5_fold(int n);       // v5 last-arriver merge: splits per load round (12 default, 4: the first version)  // split small-batch decode kernel up to n (row, kv head) pairs (0 off, <0 default)
void attn_set_v3_max_pairs(int n);  // single-workgroup-per-(row, kv head) decode kernel up to n pairs (0: off)
void attn_set_impl(int impl, int waves_target);
void attn_set_diag(int d);
void attn_set_v3_kpg(int mult);  // small-batch decode attention: key rows per lane per chunk x mult (1, 2, 4)
// bounds-checked debug build: per-translation-unit error words (JLA_BOUNDS_* bits; 0 in release builds)
unsigned jla_bounds_norm_embed(int reset);
unsigned jla_bounds_rope_kv(int reset);
unsigned jla_bounds_sample(int reset);
unsigned jla_bounds_gemm(int reset);
unsigned jla_bounds_gemv(int reset);
unsigned jla_bounds_attn_decode(int reset);
unsigned jla_bounds_attn_prefill(int reset);
int attn_decode_splits(int B, int Hkv, int T, int rep);
// ws: >= B*H*nsplit*(Dh+2) floats; tickets: B*Hkv int32, zero-initialised once (self-resetting)
int attn_decode(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const int32_t* slot, const int32_t* kv_start,
                const uint8_t* key_mask, int mask_len, bf16_t* out, float* ws, int32_t* tickets, int B, int H,
                int Hkv, int Dh, int T, int t_cap, int nsplit, hipStream_t s, bf16_t* out_pack = nullptr);
int attn_decode_packs(int B, int Hkv, int rep);
// decode attention on the matrix cores (attn_decode_mma.hip); dispatched by attn_decode (attn_set_v6 mode)
int attn_decode_v6(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const int32_t* slot, const int32_t* kv_start,
                   const uint8_t* key_mask, int mask_len, bf16_t* out, int B, int H, int Hkv, int T, int t_cap,
                   hipStream_t s, bf16_t* out_pack);
void attn_set_v6(int mode);
void attn_set_v6_wpp(int wpp);
void attn_set_v6_diag(int d);  // tools only: v6 ablations (1 no compute, 2 no K loads, 4 no V DMAs; wrong results)
int attn_v6_wpp(int pairs);
void attn_prefill_set_impl(int impl);  // 2 = GQA-shared MFMA 32x32 flash kernel (default), 1 = v1
int attn_prefill(const bf16_t* q, const bf16_t* kc, const bf16_t* vc, const int32_t* slot, const int32_t* kv_start,
                 const uint8_t* key_mask, int mask_len, bf16_t* out, int B, int S, int H, int Hkv, int Dh, int T,
                 hipStream_t s);

int argmax(const float* logits, int B, int V, int32_t* idx, float* val, hipStream_t s);
// top-k / top-p sampler (topk_sample.hip): cv/ci [B, topk_chunks(V) * K] candidates
int topk_chunks(int V);
int topk_chunk(const float* logits, int B, int V, int K, int idx_offset, float* cv, int32_t* ci, hipStream_t s);
int topk_merge(const float* cv, const int32_t* ci, int B, int C, int K, int mode, float* out_v, int32_t* out_i,
               int32_t* nxt, float temperature, float top_p, uint64_t seed, const int32_t* step, hipStream_t s);
// custom xGMI collectives over IPC-mapped uncached buffers (allreduce.hip)
size_t car_buffer_bytes(long long max_bytes, int world);
int car_alloc(long long max_bytes, int world, void** buf, void** sig, hipIpcMemHandle_t* hbuf, hipIpcMemHandle_t* hsig);
void car_free(void* buf, void* sig);
int car_init(int rank, int world, long long max_bytes, void* own_buf, void* own_sig, const hipIpcMemHandle_t* hbufs,
             const hipIpcMemHandle_t* hsigs, double timeout_s, void** state);
// op 0: out = sum over ranks of in (bf16/fp32); op 1: h (fp32) += sum, hb (bf16) = h. two_shot: reduce-scatter +
// all-gather instead of every rank reading every peer's copy
int car_reduce(void* state, int op, const void* in, void* out, float* h, bf16_t* hb, long long nbytes, int is_bf16,
               int two_shot, hipStream_t s,
               bf16_t* hb_pack = nullptr, int pack_cols = 0);
// all-gather of (fp32, int32 + idx_offset) pairs: mode 0 = first max over ranks per pair, mode 1 = [n/k][world*k]
int car_pairs(void* state, int mode, const float* a, const int32_t* b, int idx_offset, long long n, int k,
              float* out_a, int32_t* out_b, hipStream_t s);
void car_set_gran_max(long long n);  // granule one-shot up to n payload bytes per rank (0: flag protocol only)
int car_error(void* state);
const void* car_device(void* state);      // the device-side CarDevice (car.h) of an instance (MODE_TPRESID)
long long car_max_bytes(void* state);
int car_world(void* state);
int car_set_grid(void* state, int grid);  // collective blocks per launch (0: the maximum; same on every rank, before first use)
void car_destroy(void* state);
int decode_update(const int32_t* nxt, int32_t* finished, int32_t* sequences, int32_t* cur_len, int32_t* tokens,
                  int32_t* positions, int32_t* slot, int B, int L, int pad, int eos, hipStream_t s);
// CU placement (placement.hip): CU-masked streams and a census of where a launch's workgroups run
int cu_census(uint32_t* out, int blocks, hipStream_t s);
int cu_mask_stream_create(const uint32_t* mask, int words, hipStream_t* out);
int cu_mask_stream_get(hipStream_t s, uint32_t* mask, int words);
int stream_destroy(hipStream_t s);
int graph_kernel_nodes(hipGraph_t g);  // kernel nodes of a captured graph (< 0: error)

}  // namespace jla
