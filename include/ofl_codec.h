/*
 * ofl_codec.h -- C ABI of libofl_codec.so, the MI355X (gfx950) tensor-codec
 * library behind openfl_amd.pipelines.
 *
 * Every entry point is plain C: integers, sizes and raw pointers.  Device
 * pointers are HIP device addresses on the current device (e.g. a
 * torch.Tensor's data_ptr()); `stream` is a hipStream_t (e.g.
 * torch.cuda.current_stream().cuda_stream) passed as void*.  Functions return
 * 0 on success and a negative OFL_E* code on failure; ofl_last_error() then
 * returns a thread-local message.  After a plan's first use, encode/decode
 * neither allocate nor synchronise, so they are reentrant and
 * graph-capturable; concurrent calls need separate workspaces.
 *
 * The codec replaces the per-tensor Eden transformer of the reference
 * (securefederatedai/openfl v1.6, /root/reference):
 *   openfl/pipelines/eden_pipeline.py:555-611  Eden.compress     -> ofl_eden_encode
 *   openfl/pipelines/eden_pipeline.py:632-659  Eden.decompress   -> ofl_eden_decode
 *   openfl/pipelines/eden_pipeline.py:569-606  slicing rule      -> ofl_eden_slice_plan
 *   openfl/pipelines/eden_pipeline.py:771      seed `sum()` term -> ofl_serial_sum_f32/_f64
 * The Python plugin surface (EdenTransformer.forward/backward,
 * eden_pipeline.py:761-818) is mirrored by openfl_amd/pipelines/eden_pipeline.py
 * on top of these calls.  Byte layout of the output planes and the meaning of
 * every metadata value are identical to the reference's.
 */
#ifndef OFL_CODEC_H
#define OFL_CODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OFL_OK 0
#define OFL_EINVAL -1  /* bad argument (n_bits outside 1..8, dims not powers of two, ...) */
#define OFL_EHIP -2    /* a HIP runtime call failed */
#define OFL_ESPACE -3  /* workspace too small */
#define OFL_EFORMAT -4 /* input is not in the format the call handles (caller may fall back) */

/* Library version string. */
const char* ofl_version(void);

/* Thread-local message for the last failing call on this thread. */
const char* ofl_last_error(void);

/* ---- slicing rule (eden_pipeline.py:569-606) ------------------------------
 * Splits n elements into power-of-two slices: while
 * (next_po2(rem) - rem) / n > 0.1 take prev_po2(rem); the last slice takes the
 * remainder.  Each slice is padded to max(next_po2(len), 8) (:541-546).
 * Writes up to max_slices padded sizes to P_out and valid lengths to len_out
 * (either may be NULL) and returns the slice count (> max_slices means the
 * arrays were too small). */
int ofl_eden_slice_plan(int64_t n, int64_t* P_out, int64_t* len_out, int max_slices);

/* ---- plans ----------------------------------------------------------------
 * A plan describes a batch of `ntensors` fp32 tensors laid out in one fp32
 * arena (tensor t starts at element elem_offset[t] and has numel[t] elements)
 * and their Eden bit planes laid out in one byte arena (tensor t's planes
 * start at byte ofl_eden_plan_tensor_info(...).planes_offset and hold
 * n_bits * P_tot(t) / 8 bytes: plane i of tensor t is the byte range
 * [i * P_tot/8, (i+1) * P_tot/8), byte j bit b = bit i of bin[8j + b], the
 * reference's to_bits layout, eden_pipeline.py:661-690).
 *
 * slice_dims: NULL -> the reference slicing rule; otherwise nslices[t]
 * padded slice sizes per tensor, concatenated (the P_k values of a received
 * metadata dict, eden_pipeline.py:650-654).  Slice k of tensor t then holds
 * elements [sum_{k'<k} P_k', ...) truncated to numel[t] (:656-657).
 * Creating a plan is host-only (works without a GPU).  The FIRST encode or
 * decode with a plan uploads its descriptor tables (hipMalloc + one
 * synchronous copy), so that first call must not be graph-captured; later
 * calls neither allocate nor synchronise. */
typedef struct ofl_eden_plan* ofl_eden_plan_t;

int ofl_eden_plan_create(int ntensors, const int64_t* numel, const int64_t* elem_offset,
                         const int32_t* nslices, const int64_t* slice_dims, int n_bits,
                         ofl_eden_plan_t* plan_out);
void ofl_eden_plan_destroy(ofl_eden_plan_t plan);

/* Large-slice schedule (no reference counterpart: how the gfx950 passes are
 * ordered, never what they compute -- outputs are bit-identical for every
 * schedule).  Slices with P > 2^15 run in "waves" of at most wave_bytes of
 * fp32 intermediates (0: all large slices in one wave; a bigger slice is a
 * wave of its own); each wave runs all of its passes back to back and the
 * waves reuse `streams` workspace buffers, which bounds the workspace.
 * streams = 2 alternates the waves between the caller's stream and a
 * plan-owned side stream (forked from and joined back into the caller's
 * stream inside every call) so one wave's launches fill the other's launch
 * gaps and tails; there are then at least two waves (the large slices split
 * in halves).  wave_bytes < 0 or streams == 0 keep the current value.  Only
 * before the plan's first encode/decode; the workspace size changes with it.
 * Default: 2 GiB waves, 2 streams (env OFL_EDEN_WAVE_MIB / OFL_EDEN_STREAMS
 * override the default; DESIGN.md section 3.6 has the measurements). */
int ofl_eden_plan_set_schedule(ofl_eden_plan_t plan, int64_t wave_bytes, int streams);
int ofl_eden_plan_get_schedule(ofl_eden_plan_t plan, int64_t* wave_bytes, int* streams);
int ofl_eden_plan_num_waves(ofl_eden_plan_t plan);
/* Kernel choice for the large slices' row passes (no reference counterpart;
 * outputs bit-identical either way): -1 auto (launches of fewer than 5 tiles
 * per CU use the two-blocks-per-CU kernels, the rest the persistent
 * prefetching ones; env OFL_EDEN_ROW2 / OFL_EDEN_ROW2_TPC override the auto
 * rule), 0 always persistent, 1 always two blocks per CU. */
int ofl_eden_plan_set_row2(ofl_eden_plan_t plan, int mode);
/* Tile pairs in the two-blocks-per-CU row passes that apply the D1 signs
 * (encode pass A, decode pass C; no reference counterpart, outputs
 * bit-identical either way): a block runs a tile and the one 2^(p-3)
 * elements up, whose sign words are the same, and hashes them once.
 * -1 auto (launches of more tiles than two per CU; env OFL_EDEN_PAIR
 * overrides), 0 never, 1 whenever the launch holds slices of >= 2^18. */
int ofl_eden_plan_set_pair(ofl_eden_plan_t plan, int mode);
/* Launches of the tiny (<= 2^10) and small (2^11..2^15) slices (no reference
 * counterpart; outputs bit-identical either way): 1 one small-set launch of
 * 1024-thread workgroups for all of them, 0 one launch per size class, -1 the
 * default (1; env OFL_EDEN_SSET=0 selects 0).  Before the first encode/decode. */
int ofl_eden_plan_set_sset(ofl_eden_plan_t plan, int mode);
/* A plan whose large slices fit one wave and whose single-level middle passes
 * share one k_col_multi launch runs its small-set groups inside that launch,
 * on the caller's stream (no side stream, no fork / join): 1 yes, 0 the
 * small-set launch on the side stream, -1 the default (1; env
 * OFL_EDEN_FUSESET=0 selects 0).  Outputs bit-identical either way.  Before
 * the first encode/decode. */
int ofl_eden_plan_set_fuse(ofl_eden_plan_t plan, int mode);

/* Totals: slices (= length of the scales array), planes-arena bytes,
 * workspace bytes needed by encode and decode. */
int64_t ofl_eden_plan_num_slices(ofl_eden_plan_t plan);
int64_t ofl_eden_plan_planes_bytes(ofl_eden_plan_t plan);
int64_t ofl_eden_plan_workspace_bytes(ofl_eden_plan_t plan);

/* Per-tensor placement inside the arenas.  Any out pointer may be NULL. */
int ofl_eden_plan_tensor_info(ofl_eden_plan_t plan, int t, int64_t* planes_offset,
                              int64_t* planes_bytes, int32_t* first_slice, int32_t* nslices);
/* Padded size of every slice of tensor t (nslices entries). */
int ofl_eden_plan_tensor_dims(ofl_eden_plan_t plan, int t, int64_t* dims_out);

/* ---- encode / decode -------------------------------------------------------
 * seeds: DEVICE array of ntensors uint32 seeds (the metadata key 0 value,
 *        eden_pipeline.py:771-779; slices use seed and seed+1, :548-549).
 * scales: DEVICE float array of ofl_eden_plan_num_slices() entries, slice
 *        order (metadata keys 2,4,6,... :781-785).
 * Encode: x_arena (fp32, read only) -> planes_arena (every plane byte of every
 *        tensor is written) + scales.
 * Decode: planes_arena + scales -> y_arena (only the numel[t] elements of each
 *        tensor are written).
 * ws: DEVICE workspace of at least ofl_eden_plan_workspace_bytes() bytes.
 * Everything is enqueued on `stream`; nothing synchronises. */
int ofl_eden_encode(ofl_eden_plan_t plan, const float* x_arena, const uint32_t* seeds,
                    uint8_t* planes_arena, float* scales, void* ws, size_t ws_bytes,
                    void* stream);
int ofl_eden_decode(ofl_eden_plan_t plan, const uint8_t* planes_arena, const uint32_t* seeds,
                    const float* scales, float* y_arena, void* ws, size_t ws_bytes,
                    void* stream);
/* encode fused with the aggregator's WeightedAverage + generate_delta
 * (aggregator.py:780-865, weighted_average.py:14, tensor_codec.py:150-180):
 * the large slices' row pass computes x = float32((sum_c f64(x_c) * w_c) /
 * wsum - f64(base)) from the ncollab (1..16) collaborator arenas (device array
 * collab_arenas of device pointers, weights a DEVICE float64 array; arenas,
 * base_arena (nullable) and delta_arena share the plan's layout) instead of
 * reading a delta arena -- the delta's 8 B/element round trip through HBM
 * is not made.  Slices of at most 2^15 elements still read delta_arena, so
 * the caller fills it for their ranges (ofl_wavg_delta_ranges32).  Outputs
 * equal ofl_eden_encode of the delta ofl_wavg_delta would write. */
int ofl_eden_encode_wavg(ofl_eden_plan_t plan, const float* const* collab_arenas, const double* weights,
                         int ncollab, double wsum, const float* base_arena, const float* delta_arena,
                         const uint32_t* seeds, uint8_t* planes_arena, float* scales, void* ws, size_t ws_bytes,
                         void* stream);
/* decode fused with TensorCodec.apply_delta (tensor_codec.py:182-211):
 * y = base + decoded, two float32 roundings as in NumPy (decoded delta first,
 * then the add).  base_arena has the plan's layout; y_arena may alias it. */
int ofl_eden_decode_add(ofl_eden_plan_t plan, const uint8_t* planes_arena, const uint32_t* seeds,
                        const float* scales, const float* base_arena, float* y_arena, void* ws,
                        size_t ws_bytes, void* stream);

/* The one-tensor plugin path (Eden.compress / Eden.decompress,
 * eden_pipeline.py:555-659, one tensor per TensorCodec call) in one native
 * call: one H2D of a pinned host block, the launches, one D2H of a device
 * block, then a synchronize of `stream` -- no per-copy runtime calls from the
 * caller.  Encode input block (in_host pinned -> in_dev, in_bytes): x arena
 * at 0, seeds (uint32 per tensor) at off_seeds >= 4 * arena length; output
 * block (out_dev -> out_host, out_bytes): planes arena at 0, scales (fp32 per
 * slice) at off_scales >= planes bytes.  Decode input block: planes arena at
 * 0, scales at off_scales, seeds at off_seeds; output block: the y arena
 * (out_bytes <= 4 * arena length copied back). */
/* Zero-copy variants for plans of tiny / small slices only (every slice <=
 * 2^15 elements; else OFL_EINVAL): the same blocks, but in_host / out_host /
 * y_host are MAPPED pinned host memory (hipHostMalloc, torch pin_memory) that
 * the single launch reads and writes directly -- no DMA copies; y_host holds
 * 4 * arena bytes.  Synchronous (stream synchronised).  Not mapped -> OFL_EINVAL. */
/* Second half of a one-tensor encode whose x is already on (or on its way
 * to) the device, e.g. by ofl_copy_h2d_chunked on the same stream: the seed
 * written into in_dev + off_seeds, the launches, one D2H of [planes | scales]
 * into out_host (pinned), stream synchronised. */
int ofl_eden_encode_seeded(ofl_eden_plan_t plan, void* in_dev, size_t off_seeds, uint32_t seed, void* out_dev,
                           void* out_host, size_t out_bytes, size_t off_scales, void* ws, size_t ws_bytes, void* stream);
int ofl_eden_encode_mapped(ofl_eden_plan_t plan, const void* in_host, size_t off_seeds, void* out_host,
                           size_t off_scales, void* ws, size_t ws_bytes, void* stream);
int ofl_eden_decode_mapped(ofl_eden_plan_t plan, const void* in_host, size_t off_scales, size_t off_seeds,
                           void* y_host, void* ws, size_t ws_bytes, void* stream);
int ofl_eden_encode_host(ofl_eden_plan_t plan, const void* in_host, void* in_dev, size_t in_bytes, size_t off_seeds,
                         void* out_dev, void* out_host, size_t out_bytes, size_t off_scales, void* ws, size_t ws_bytes,
                         void* stream);
int ofl_eden_decode_host(ofl_eden_plan_t plan, const void* in_host, void* in_dev, size_t in_bytes, size_t off_scales,
                         size_t off_seeds, void* out_dev, void* out_host, size_t out_bytes, void* ws, size_t ws_bytes,
                         void* stream);
/* The same one-tensor calls for large tensors, the host buffers used where
 * they lie (pageable is fine; the runtime streams them at the pinned rate on
 * this box) instead of being copied into a pinned block first:
 *   encode_host_x: x_host (x_bytes, NULL = already copied to in_dev, e.g. by
 *     ofl_copy_h2d_async while the host computed the seed's serial sum),
 *     the seed written to in_dev + off_seeds by a device memset;
 *   decode_host_x: planes and scales from separate host arrays, the seed by
 *     a device memset, y D2H into y_host.
 * Both synchronise `stream` before returning. */
int ofl_eden_encode_host_x(ofl_eden_plan_t plan, const void* x_host, size_t x_bytes, uint32_t seed, void* in_dev,
                           size_t off_seeds, void* out_dev, void* out_host, size_t out_bytes, size_t off_scales,
                           void* ws, size_t ws_bytes, void* stream);
int ofl_eden_decode_host_x(ofl_eden_plan_t plan, const void* planes_host, size_t planes_bytes, const float* scales_host,
                           int nscales, uint32_t seed, void* in_dev, size_t off_scales, size_t off_seeds,
                           void* out_dev, void* y_host, size_t y_bytes, void* ws, size_t ws_bytes, void* stream);
/* hipMemcpyAsync host -> device on `stream` (no synchronisation). */
int ofl_copy_h2d_async(void* dst_dev, const void* src_host, size_t bytes, void* stream);
/* The same copy from PAGEABLE host memory (a received payload), staged: the
 * bytes go in 4 MiB chunks through a library-owned pinned ring on up to
 * nthreads (<= 8) host threads, each chunk's async H2D on `stream` issued as
 * soon as it is staged, so the host copies and the DMAs run together.
 * Returns when every chunk is staged and enqueued: the source may be
 * released then, and work enqueued on `stream` afterwards sees the data.
 * Each device keeps up to 4 rings (concurrent callers each take one, a fifth
 * waits); copies under 8 MiB go straight to hipMemcpyAsync. */
int ofl_copy_h2d_staged(void* dst_dev, const void* src_host, size_t bytes, int nthreads, void* stream);
/* The current device's side stream `index` (0..2), created once per device,
 * all three together: the Eden plans' side streams and the pipelined
 * inflate's piece streams (1, 2).  HIP gives streams the GPU_MAX_HW_QUEUES
 * hardware queues in turn and streams on one queue run in order, so the
 * library shares these instead of making more. */
int ofl_side_stream(int index, void** stream);

/* ---- profiling (bench.py) --------------------------------------------------
 * While enabled, every encode/decode of the plan records a HIP event before
 * and after each launch, on the launch's stream.  collect() waits for
 * the recorded calls of one direction, writes the summed per-launch
 * milliseconds (launch order) and the call count, and drops the records.
 * launch_info() names launch idx (kernel symbol as rocprofv3 shows it) with
 * its grid size, the bytes it reads+writes in HBM and its share of the
 * algorithmic bytes (input/output fp32 + bit planes; FWHT intermediates 0). */
int ofl_eden_plan_profile(ofl_eden_plan_t plan, int enable);
int ofl_eden_plan_num_launches(ofl_eden_plan_t plan, int encode);
int ofl_eden_plan_launch_info(ofl_eden_plan_t plan, int encode, int idx, char* name, int cap,
                              int64_t* blocks, int64_t* bytes_moved, int64_t* bytes_alg);
int ofl_eden_plan_profile_collect(ofl_eden_plan_t plan, int encode, double* ms_sum, int max,
                                  int* ncalls);

/* ---- lossy k-means / sparsify / ternary pipelines ---------------------------
 * (openfl/pipelines/kc_pipeline.py, skc_pipeline.py, stc_pipeline.py).  Device
 * pointers as above; scalar results come back in host memory, so these calls
 * synchronise `stream`.  ws: DEVICE scratch of ofl_lossy_workspace_bytes(n).
 *
 * ofl_kmeans1d_fit   replaces sklearn KMeans(n_clusters=k, n_init).fit on a
 *                    column vector (kc_pipeline.py:49-56, skc_pipeline.py:127-131):
 *                    sorted centres, per-cluster counts, inertia.
 * ofl_kmeans1d_label labels as float32 values: out[i] = rank_of_cluster[c(i)],
 *                    c(i) = nearest centre (np.choose + _float_to_int, :55-61, :88-114)
 * ofl_sparsify_topk  SparsityTransformer.forward (skc_pipeline.py:33-54,72-94):
 *                    keep the k largest |x| (ties: lowest index), +1e-7 shift rule,
 *                    dense float32 output + kept-set statistics
 * ofl_ternary_stats  TernaryTransformer.forward mean/sign counts (stc_pipeline.py:120-123)
 * ofl_ternary_ranks  TernaryTransformer.forward ranks (stc_pipeline.py:105-130)
 * ofl_lut_decode     the sequential in-place key->value replacement of every
 *                    lossy backward (kc_pipeline.py:81-83, stc_pipeline.py:139-142) */
const char* ofl_lossy_last_error(void);
size_t ofl_lossy_workspace_bytes(int64_t n);
int ofl_kmeans1d_fit(const float* x, int64_t n, int k, int n_init, uint64_t seed, int max_exact,
                     double* centres, int64_t* counts, double* inertia, void* ws, size_t ws_bytes,
                     void* stream);
/* Batched, device-resident 1-D k-means (KmeansTransformer.forward for many
 * tensors at once, kc_pipeline.py:47-63 / skc_pipeline.py:127-131): tensor t
 * is x_arena[offsets[t], offsets[t] + numels[t]) (host arrays; numels[t] >= k).
 * Per tensor: min/max, 4096-bin histogram, weighted k-means++ (2 + ln k local
 * trials, n_init restarts) + Lloyd on the histogram, then up to max_exact + 1
 * exact Lloyd passes over the data until the float32 midpoints stop moving.
 * ranks_out (device, same layout, may be NULL): float32 rank of each element's
 * cluster among np.unique(used centres as value dtype: float64 if value_f64,
 * else float32) -- the GZIPTransformer input.  Host outputs (any may be NULL):
 * centres / counts / uniq [ntensors * k] (sorted), inertia / nuniq [ntensors].
 * Deterministic (integer atomics, fixed-order reductions); one sync at the end. */
size_t ofl_kmeans1d_batch_workspace_bytes(int ntensors, const int64_t* numels);
int ofl_kmeans1d_batch(int ntensors, const float* x_arena, const int64_t* offsets, const int64_t* numels, int k,
                       int n_init, uint64_t seed, int max_exact, int value_f64, float* ranks_out, double* centres,
                       int64_t* counts, double* inertia, int32_t* nuniq, double* uniq, void* ws, size_t ws_bytes,
                       void* stream);
/* One tensor's labelling rule after ofl_kmeans1d_batch (k <= 8): an element
 * x of [start, end) is labelled rank[j] for the first j with x <= mid[j]
 * (mid[j] = float32 midpoint of sorted centres j and j + 1, +inf from k - 1
 * on) -- the ranks ranks_out receives.  ofl_gzip_label_to reads these
 * records instead of a rank array. */
typedef struct {
    int64_t start, end;  /* arena element range */
    float mid[8];
    float rank[8];
} ofl_label_rec;
/* ofl_kmeans1d_batch that also writes label_tab (DEVICE, ntensors records,
 * ascending non-overlapping ranges required; k <= 8), e.g. with ranks_out
 * NULL, so that the rank array is never written (ofl_gzip_label_to). */
int ofl_kmeans1d_batch_tab(int ntensors, const float* x_arena, const int64_t* offsets, const int64_t* numels, int k,
                           int n_init, uint64_t seed, int max_exact, int value_f64, float* ranks_out,
                           ofl_label_rec* label_tab, double* centres, int64_t* counts, double* inertia,
                           int32_t* nuniq, double* uniq, void* ws, size_t ws_bytes, void* stream);
int ofl_kmeans1d_label(const float* x, int64_t n, const double* centres, int k,
                       const float* rank_of_cluster, float* out, void* stream);
int ofl_sparsify_topk(const float* x, int64_t n, int64_t k, float* sparse_out, float* kept_min,
                      int64_t* n_pos, int64_t* n_neg, int64_t* n_zero, double* abs_sum, int* shifted,
                      void* ws, size_t ws_bytes, void* stream);
/* ofl_sparsify_topk for many tensors of one arena (tensor t at offsets[t],
 * numels[t] elements, keep ks[t] with 1 <= ks[t] <= numels[t]; host arrays).
 * Radix select on the device (3 digit passes + tie pass + select pass, no
 * host round trips); sparse_arena (device, same layout) gets the dense
 * float32 sparse output.  Host outputs [ntensors] (any may be NULL) as in
 * ofl_sparsify_topk.  Deterministic; one sync at the end.
 * ws: ofl_sparsify_topk_batch_workspace_bytes(). */
size_t ofl_sparsify_topk_batch_workspace_bytes(int ntensors, const int64_t* numels);
int ofl_sparsify_topk_batch(int ntensors, const float* x_arena, const int64_t* offsets, const int64_t* numels,
                            const int64_t* ks, float* sparse_arena, float* kept_min, int64_t* n_pos, int64_t* n_neg,
                            int64_t* n_zero, double* abs_sum, int32_t* shifted, void* ws, size_t ws_bytes,
                            void* stream);
int ofl_ternary_stats(const float* x, int64_t n, int64_t* n_pos, int64_t* n_neg, double* abs_sum, void* ws,
                      size_t ws_bytes, void* stream);
int ofl_ternary_ranks(const float* sparse, int64_t n, float rank_neg, float rank_zero, float rank_pos,
                      float* out, void* stream);
/* ofl_ternary_ranks for many tensors of one arena: ranks3[3 t .. 3 t + 2] =
 * (rank_neg, rank_zero, rank_pos) of tensor t (host, copied before return).
 * ws: ofl_ternary_ranks_batch_workspace_bytes(). */
size_t ofl_ternary_ranks_batch_workspace_bytes(int ntensors);
int ofl_ternary_ranks_batch(int ntensors, const float* sparse_arena, const int64_t* offsets, const int64_t* numels,
                            const float* ranks3, float* out_arena, void* ws, size_t ws_bytes, void* stream);
int ofl_lut_decode(const float* in, int64_t n, const float* keys, const float* vals, int nk, float* out,
                   void* stream);
/* ofl_lut_decode for many tensors of one arena in one launch: tensor t has
 * nk[t] <= max_nk <= 64 keys at keys[t * max_nk ...] (host arrays, copied
 * before the call returns); ws: ofl_lut_decode_batch_workspace_bytes(). */
size_t ofl_lut_decode_batch_workspace_bytes(int ntensors, int max_nk);
int ofl_lut_decode_batch(int ntensors, const float* in_arena, const int64_t* offsets, const int64_t* numels,
                         const int32_t* nk, const float* keys, const float* vals, int max_nk, float* out_arena,
                         void* ws, size_t ws_bytes, void* stream);

/* ---- aggregator end of round (csrc/agg_kernels.hip) -------------------------
 * Aggregator._prepare_trained (aggregator.py:780-865) runs, per tensor,
 * WeightedAverage (weighted_average.py:12-14, np.average(tensors, weights,
 * axis=0)), TensorCodec.generate_delta (tensor_codec.py:150-180: new - base),
 * compress + decompress, and apply_delta (tensor_codec.py:182-211: base +
 * delta).  These entry points do the arithmetic on flat device arenas
 * (all tensors of a model update), bit-exact with NumPy: float64 products and
 * an in-order float64 sum over collaborators, division by wsum (the float64
 * sum of the weights, computed by the caller with NumPy), float64 subtraction
 * of the float32 base.  Errors: ofl_agg_last_error().
 *
 * ofl_wavg_delta  xs: host array of ncollab device pointers (n floats each),
 *                 weights: host [ncollab].  base may be NULL (delta = average).
 *                 Outputs (device, any may be NULL): agg_out float64 average
 *                 (required as running sums when ncollab > 16), delta64_out
 *                 float64 delta, delta32_out the delta rounded to float32 (the
 *                 codec input, Eden.compress :579).
 * ofl_wavg_delta_ranges  the float64 delta at listed element ranges (host
 *                 starts/counts; single[r] != 0: a single-element tensor,
 *                 pairwise order as below), packed into out (device) -- the
 *                 values the Eden seed's serial sums read.  Synchronous.
 * ofl_wavg_delta_range_sums  the same ranges, each summed left to right in
 *                 float64 on the device (Python's sum() of the seed formula,
 *                 eden_pipeline.py:771); sums: host [nranges].  Synchronous.
 * ofl_wavg_delta_points  recompute listed elements (host idx) the way NumPy
 *                 reduces a single-element tensor's (C, 1) stack: pairwise
 *                 sum of the C products (1 <= ncollab <= 2048);
 *                 call after ofl_wavg_delta for the 1-element tensors.
 * ofl_apply_delta out = base + delta in float32 (out may alias either input).
 * ofl_apply_delta_ranges  the same on listed ranges; starts [nranges] and dst
 *                 [nranges + 1] (exclusive prefix of the range lengths, dst[n]
 *                 = total) are DEVICE arrays, so nothing synchronises. */
const char* ofl_agg_last_error(void);
int ofl_wavg_delta(int ncollab, const float* const* xs, const double* weights, double wsum, const float* base,
                   int64_t n, double* agg_out, double* delta64_out, float* delta32_out, void* stream);
size_t ofl_wavg_ranges_workspace_bytes(int ncollab, int nranges);
int ofl_wavg_delta_ranges(int ncollab, const float* const* xs, const double* weights, double wsum,
                          const float* base, int nranges, const int64_t* starts, const int64_t* counts,
                          const int32_t* single, double* out, void* ws, size_t ws_bytes, void* stream);
size_t ofl_wavg_range_sums_workspace_bytes(int ncollab, int nranges, int64_t total);
int ofl_wavg_delta_range_sums(int ncollab, const float* const* xs, const double* weights, double wsum,
                              const float* base, int nranges, const int64_t* starts, const int64_t* counts,
                              const int32_t* single, double* sums, void* ws, size_t ws_bytes, void* stream);
/* ofl_wavg_delta_seeds  the Eden seeds of a round end without a host round
 *                 trip: the float64 delta on the listed ranges (packed_dev,
 *                 total doubles), their left-to-right sums (sums_dev), and
 *                 seeds_dev[r] = (hash(sum*13 + 7) + draws_dev[r]) % 2^16 with
 *                 CPython's float hash (eden_pipeline.py:771-772).  Every
 *                 pointer is DEVICE memory (xs_dev: ncollab pointers,
 *                 weights_dev, starts_dev [nranges], dst_dev [nranges + 1]
 *                 prefix of the range lengths, single_dev [nranges]).  Async.
 * ofl_py_hash_doubles  CPython's hash() of n device doubles (NaN -> 0). */
int ofl_wavg_delta_seeds(int ncollab, const float* const* xs_dev, const double* weights_dev, double wsum,
                         const float* base, int nranges, const int64_t* starts_dev, const int64_t* dst_dev,
                         const int32_t* single_dev, int64_t total, const int64_t* draws_dev, uint32_t* seeds_dev,
                         double* sums_dev, double* packed_dev, void* stream);
int ofl_py_hash_doubles(const double* v_dev, int n, int64_t* out_dev, void* stream);
size_t ofl_wavg_points_workspace_bytes(int ncollab, int npoints);
int ofl_wavg_delta_points(int ncollab, const float* const* xs, const double* weights, double wsum, const float* base,
                          int npoints, const int64_t* idx, double* agg_out, double* delta64_out, float* delta32_out,
                          void* ws, size_t ws_bytes, void* stream);
int ofl_apply_delta(const float* base, const float* delta, int64_t n, float* out, void* stream);
/* out = (double)data - shift in float64 (device arrays): RandomShiftTransformer.backward
 * (random_shift_pipeline.py:45-68) with float64 shifts (metadata off the wire);
 * its forward (data + shift, float32) is ofl_apply_delta. */
int ofl_sub_f32_f64(const float* data, const double* shift, int64_t n, double* out, void* stream);
int ofl_apply_delta_ranges(const float* base, const float* delta, float* out, int nranges, const int64_t* starts,
                           const int64_t* dst, int64_t total, void* stream);
/* ofl_wavg_delta's float32 delta on listed ranges only (xs: host array of
 * ncollab <= 16 device pointers; starts [nranges] / dst [nranges + 1]: DEVICE
 * tables as ofl_apply_delta_ranges): what ofl_eden_encode_wavg reads. */
int ofl_wavg_delta32_ranges(int ncollab, const float* const* xs, const double* weights, double wsum,
                            const float* base, int nranges, const int64_t* starts, const int64_t* dst, int64_t total,
                            float* delta32_out, void* stream);

/* ---- gzip of rank arrays (csrc/deflate_kernels.hip) -------------------------
 * GZIPTransformer.forward (kc_pipeline.py:128-141, skc_pipeline.py:201-215,
 * stc_pipeline.py:185-199) compresses the float32 ranks with gzip.compress;
 * GZIPTransformer.backward (kc_pipeline.py:152-156) is gzip.decompress, which
 * reads any valid stream.  ofl_gzip_ranks produces one on the GPU (TLZ): a
 * multi-member gzip stream, one member per 131072 float32 values (512 KiB),
 * each ONE dynamic-Huffman deflate block over the full 32 KiB window whose
 * copies are whole values (3..64 values at distances of 4-byte multiples),
 * chosen by an optimal parse (0.115 of the input on KC ranks; gzip -9: 0.117);
 * CRC-32 and ISIZE per member.  Every member header carries an RFC 1952 extra
 * subfield 'OZ': version 1, log2 of the segment length (11), the segment
 * count, the member's byte size, its value count and, per segment of 2048
 * values, the bit offset of its first symbol (no copy crosses a segment end),
 * which gzip.decompress skips.  x: DEVICE float32 [n], every value an integer
 * 0..31 (the ranks the lossy pipelines write; anything else -> OFL_EINVAL,
 * nothing written).  out: HOST buffer of out_cap >= ofl_gzip_ranks_bound(n)
 * bytes; *out_len = stream length.  When out is mapped pinned memory
 * (hipHostMalloc, torch pin_memory) each batch of members is packed into
 * device staging and crosses PCIe by one DMA while the next batch encodes;
 * pageable memory gets one synchronous D2H per batch.  ws: device,
 * ofl_gzip_ranks_workspace_bytes(n).
 * Synchronous.  Deterministic (the header's mtime is 0).  Errors:
 * ofl_gzip_last_error(). */
const char* ofl_gzip_last_error(void);
size_t ofl_gzip_ranks_workspace_bytes(int64_t n);
size_t ofl_gzip_ranks_bound(int64_t n);
int ofl_gzip_ranks(const float* x, int64_t n, uint8_t* out, size_t out_cap, size_t* out_len, void* ws,
                   size_t ws_bytes, void* stream);
/* ofl_gzip_ranks that also leaves the stream in host_dst (HOST, pageable,
 * host_cap >= out_cap bytes, e.g. the payload object's own buffer): each
 * batch's bytes are copied out of `out` on nthreads host threads as soon as
 * its DMA completes, while the next batch encodes, so only the last batch's
 * copy follows the GPU work (GZIPTransformer.forward returns a fresh bytes,
 * kc_pipeline.py:128-141). */
int ofl_gzip_ranks_to(const float* x, int64_t n, uint8_t* out, size_t out_cap, uint8_t* host_dst, size_t host_cap,
                      int nthreads, size_t* out_len, void* ws, size_t ws_bytes, void* stream);
/* The k-means labelling fused into the encoder: x is the VALUE arena the
 * k-means ran on and every value is labelled through label_tab (DEVICE,
 * ntensors ofl_label_rec from ofl_kmeans1d_batch_tab) as it is loaded, so the
 * stream equals ofl_gzip_ranks_to of the ranks ranks_out would hold (0 for
 * elements outside every range).  host_dst may be NULL (then as
 * ofl_gzip_ranks). */
int ofl_gzip_label_to(const float* x, int64_t n, const ofl_label_rec* label_tab, int ntensors, uint8_t* out,
                      size_t out_cap, uint8_t* host_dst, size_t host_cap, int nthreads, size_t* out_len, void* ws,
                      size_t ws_bytes, void* stream);
/* GZIPTransformer.backward (kc_pipeline.py:152-156: gzip.decompress) for a
 * stream whose members all carry a size field ('OZ', or BGZF's 'BC'):
 * members are located from their headers and inflated (zlib) on nthreads host
 * threads into dst (HOST, cap bytes; NULL: only *out_len = decompressed
 * size), with each member's ISIZE and CRC-32 checked.  OFL_EFORMAT if the
 * stream is not member-indexed (e.g. gzip.compress output): use
 * gzip.decompress then. */
int ofl_gunzip_members(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len, int nthreads);
/* The same decode on the GPU, in two steps.  ofl_gzip_member_index (HOST, no
 * GPU): the members of a member-indexed stream src[n] (OFL_EFORMAT otherwise)
 * -> *nmembers, *out_len (decompressed size), *max_isize, *all_tlz (every
 * member carries a valid 'OZ' table; nullable) and, when index is not NULL
 * (cap_members entries), per member four int64: deflate data offset, data
 * length (| 1 << 62 for a TLZ member), output offset, ISIZE | CRC-32 << 32.
 * ofl_inflate_tlz (all members TLZ): k_tlz_ops -- one wavefront per member,
 * one lane per segment, Huffman decode from the segment's bit offset, op
 * records written over the segment's own output bytes -- then k_tlz_resolve
 * -- one block per member: op positions, every value's source by pointer
 * jumping in LDS, the float32 values, CRC-32 and ISIZE checked; data the TLZ
 * decoder does not expect goes through ofl_inflate_members instead (which
 * decides whether it is valid deflate).  ws: DEVICE,
 * ofl_inflate_tlz_workspace_bytes(nmembers).  ofl_inflate_members: any
 * member-indexed deflate data (one wavefront per member; stored, fixed and
 * dynamic blocks); ws: DEVICE, >= 256 bytes.  Both: src is the DEVICE copy
 * of the stream, readable for 32 bytes past its end; out DEVICE, out_cap
 * bytes, every member at its output offset; index the DEVICE copy of the
 * index.  Synchronous; OFL_EINVAL for corrupt data (what gzip.decompress
 * would raise on). */
int ofl_gzip_member_index(const uint8_t* src, size_t n, int64_t* index, int64_t cap_members, int64_t* nmembers,
                          size_t* out_len, uint32_t* max_isize, int* all_tlz);
size_t ofl_inflate_tlz_workspace_bytes(int64_t nmembers);
int ofl_inflate_tlz(const uint8_t* src, const int64_t* index, int64_t nmembers, uint8_t* out, size_t out_cap, void* ws,
                    size_t ws_bytes, void* stream);
/* ofl_inflate_tlz in pieces, so the pieces' H2D can overlap the inflate of
 * earlier ones: _async launches members [first, first + count) of the index
 * (no synchronisation; first == 0 also resets the status word), _wait
 * synchronises the stream, checks every launched member and, if the TLZ
 * decoder refused any, runs ofl_inflate_members over all nmembers. */
int ofl_inflate_tlz_async(const uint8_t* src, const int64_t* index, int64_t first, int64_t count, uint8_t* out,
                          size_t out_cap, void* ws, size_t ws_bytes, void* stream);
int ofl_inflate_tlz_wait(const uint8_t* src, const int64_t* index, int64_t nmembers, uint8_t* out, size_t out_cap,
                         void* ws, size_t ws_bytes, void* stream);
/* ofl_inflate_tlz_async without the status reset: pieces launched on several
 * streams as their bytes land (the caller resets the status once, e.g. with
 * ofl_inflate_tlz_async(first = 0, count = 0), orders every piece after it
 * and joins the streams before ofl_inflate_tlz_wait). */
int ofl_inflate_tlz_launch(const uint8_t* src, const int64_t* index, int64_t first, int64_t count, uint8_t* out,
                           size_t out_cap, void* ws, size_t ws_bytes, void* stream);
/* The KC backward fused (kc_pipeline.py:152-156 then :65-86): the same
 * launch, but the values stored are lut_tab[t * 32 + rank] for the element's
 * tensor t, tensors being the element ranges [lut_start[t], lut_end[t]) of the
 * float32 output (sorted, disjoint; device arrays); elements between tensors
 * store the rank.  lut_tab[t] is the tensor's int_to_float map applied to
 * every rank 0..31 in the reference's sequential order.  Finish with
 * ofl_inflate_tlz_check, which returns OFL_EFORMAT where the TLZ decoder
 * refused a member (the caller then runs ofl_inflate_members and the LUT
 * itself; no fallback runs inside). */
int ofl_inflate_tlz_launch_lut(const uint8_t* src, const int64_t* index, int64_t first, int64_t count, uint8_t* out,
                               size_t out_cap, void* ws, size_t ws_bytes, const float* lut_tab, const int64_t* lut_start,
                               const int64_t* lut_end, int32_t lut_n, void* stream);
int ofl_inflate_tlz_check(int64_t nmembers, void* ws, size_t ws_bytes, void* stream);
int ofl_inflate_members(const uint8_t* src, const int64_t* index, int64_t nmembers, uint32_t max_isize, uint8_t* out,
                        size_t out_cap, void* ws, size_t ws_bytes, void* stream);
/* Per-kernel timing of the gzip / inflate launches (bench.py): enable (1)
 * resets and starts recording HIP events around every launch of this
 * process's calls, 0 stops; collect synchronises the recorded events and
 * returns, per kernel name (newline-separated in names), the summed
 * milliseconds and the launch count, then clears the record. */
int ofl_gzip_profile(int enable);
int ofl_gzip_profile_collect(char* names, size_t names_cap, double* ms, int64_t* launches, int max_kernels,
                             int* nkernels);

/* ---- host helpers ----------------------------------------------------------
 * Left-to-right serial sums in the array's own precision: the
 * `sum(data.flatten())` term of the reference seed formula
 * (eden_pipeline.py:771, NumPy scalar arithmetic).  Host pointers. */
float ofl_serial_sum_f32(const float* x, int64_t n);
double ofl_serial_sum_f64(const double* x, int64_t n);
/* The same float32 chain, exact, on up to nthreads threads (<= 0: env
 * OFL_SUM_THREADS, default 8) -- binade-wise integer prefix sums stitched in
 * order (csrc/serial_sum.cpp); dst (or NULL) receives a copy of x.
 * ofl_serial_sum_f32, ofl_serial_sum_copy_f32 and ofl_copy_h2d_chunked use it
 * from 2^20 elements. */
float ofl_serial_sum_f32_mt(const float* x, int64_t n, float* dst, int nthreads);
/* ofl_serial_sum_f32 of x while copying x to dst (the pinned staging block
 * of a one-tensor encode): the copy rides in the add chain's latency. */
float ofl_serial_sum_copy_f32(const float* x, float* dst, int64_t n);
/* x (pageable host float32[n]) -> pinned staging -> device, in chunks of
 * `chunk` elements: each chunk's async H2D on `stream` is issued as soon as it
 * sits in the pinned buffer, so the DMA runs beside the copy of the next one
 * (and, want_sum != 0, beside the reference seed's serial float32 sum, one
 * dependent chain over all chunks: *sum_out = ofl_serial_sum_f32(x, n)).
 * The caller keeps `pinned` alive until the stream has passed the copies. */
int ofl_copy_h2d_chunked(const float* x, float* pinned, void* dev, int64_t n, int64_t chunk, int want_sum,
                         float* sum_out, void* stream);
/* ofl_serial_sum_* of n host arrays (f32 or, if f64, double) on up to
 * nthreads native threads, largest first; out[i] as double (exact for f32). */
int ofl_serial_sums_many(int n, const void* const* ptrs, const int64_t* lens, int f64, double* out, int nthreads);
/* n host memcpy's (dst[i] <- src[i], bytes[i]) on up to nthreads threads, the
 * bytes split evenly: the staging fills and output copies of the batched
 * pipeline calls (GIL-free from ctypes). */
int ofl_host_copy_many(int n, void* const* dst, const void* const* src, const int64_t* bytes, int nthreads);

#ifdef __cplusplus
}
#endif
#endif /* OFL_CODEC_H */
