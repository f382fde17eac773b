/*
 * lgcn.h — C ABI of liblgcn.so, the MI355X (gfx950) LightGCN propagation library.
 *
 * This is the drop-in boundary for the reference's hot path: K-layer LightGCN message
 * passing, i.e. torch_geometric.nn.LGConv (PyG 2.4.0) called once per layer from
 * LightGCN.forward (reference models/light_gcn.py:24,32-34), plus the gradient that
 * autograd takes through it during utils/train_test.py:train (reference
 * utils/train_test.py:90-96).
 *
 * The reference has no FFI of its own (it is pure Python over PyG/ATen); the entry points
 * below are exactly what a ctypes binding of this path needs (INTEGRATION.md shows it):
 * plain pointers, sizes and a HIP stream, no torch types.
 *
 * Conventions
 *   - Every function returns 0 on success, a positive hipError_t on a HIP failure, or a
 *     negative LGCN_E_* code on an argument error; lgcn_last_error() describes the last
 *     failure on the calling thread.
 *   - The library never allocates or frees device memory and never synchronises: the
 *     caller owns every buffer (including workspaces) and all work is ordered on the
 *     caller's stream, so every call is hipGraph-capturable.
 *   - Node ids are int64 on input (as edge_index is LongTensor[2,E] in the reference);
 *     inside a plan they are int32 (N < 2^31) and CSR offsets are int64.
 *   - Embedding tables are row-major fp32 [rows, d]. A "split" table is two pointers
 *     (lo, hi) and a split row S: row r lives at lo + r*d when r < S, else at
 *     hi + (r - S)*d. This lets layer 0 read user_embedding.weight and
 *     item_embedding.weight in place instead of materialising torch.cat
 *     (reference models/light_gcn.py:29).
 */
#ifndef LGCN_H
#define LGCN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* lgcn_stream_t; /* a hipStream_t; NULL = the null stream */

#define LGCN_ABI_VERSION 11

#define LGCN_OK 0
#define LGCN_E_ARG (-1)         /* bad size / null pointer / unsupported argument */
#define LGCN_E_WORKSPACE (-2)   /* workspace smaller than lgcn_*_workspace_size() said */
#define LGCN_E_UNSUPPORTED (-3) /* d or E outside what the kernels handle */

/* One load-balanced unit of propagation work: edges [beg, beg+len) of one CSR row.
 * dst >= 0: the whole row, write the epilogue for row dst.
 * dst <  0: one chunk of a split row, write its partial sum to partial slot (-dst-1). */
typedef struct {
    int64_t beg;
    int32_t len;
    int32_t dst;
} lgcn_item_t;

/* A row whose edges were split into pcnt chunks; partials pbeg..pbeg+pcnt-1 (in edge order). */
typedef struct {
    int32_t row;
    int32_t pbeg;
    int32_t pcnt;
    int32_t pad;
} lgcn_split_t;

/* Epilogue modes of lgcn_spmm. v = sum over the row's edges of val[e] * x[col[e]],
 * accumulated sequentially in CSR order (the order CPU scatter_add_ uses).
 *   INIT : y[r] = v (if y);  acc[r] = e[r] + v
 *   ADD  : y[r] = v (if y);  acc[r] = acc[r] + v
 *   FINAL_ACC : acc[r] = ((acc[r] + v) / div) * mul
 *   FINAL_E   : acc[r] = ((e[r]  + v) / div) * mul
 *   STORE     : acc[r] = v   (a bare LGConv layer)
 *   SCALE     : acc[r] = (v * mul) / div   (the backward seed from summed gradient rows)
 * LightGCN forward with K layers (reference models/light_gcn.py:29-36):
 *   layer 1 INIT(e=x0), layers 2..K-1 ADD, layer K FINAL_ACC(div=K+1, mul=fp32(1/(K+1)));
 *   K == 1 uses FINAL_E(e=x0).
 * Backward (autograd of the same): g = (dF*mul)/div, then K times INIT(e=g) over the
 * transposed plan. */
enum {
    LGCN_EPI_INIT = 0,
    LGCN_EPI_ADD = 1,
    LGCN_EPI_FINAL_ACC = 2,
    LGCN_EPI_FINAL_E = 3,
    LGCN_EPI_STORE = 4,
    LGCN_EPI_SCALE = 5
};

const char* lgcn_last_error(void);
int lgcn_abi_version(void);
/* sha256 (hex) of the sources this library was compiled from: every csrc translation unit,
 * lgcn_common.h and this header (build provenance; lgcn_amd._ffi refuses a mismatch). */
const char* lgcn_source_sha256(void);

/* 128-bit content digest of nbytes at data (ABI 9), on the device: out[0..1] (device uint64[2])
 * from two independent sums mod 2^64 of keyed murmur3-fmix64 mixes of the 8-byte words and their
 * positions (the < 8 trailing bytes as one more word), the length folded in — deterministic, order
 * sensitive. ws: device uint64[>= 2 * LGCN_DIGEST_BLOCKS]; data 8-byte aligned. Stream-ordered, no
 * sync. Replaces the host copy + XXH3 with which lgcn_amd._cache keyed a device edge_index by
 * content (the per-batch caches behind reference data/dataset_handler.py:285's loader, which
 * collates new tensors every epoch). */
#define LGCN_DIGEST_BLOCKS 1024
int lgcn_digest128(const void* data, int64_t nbytes, uint64_t* ws, int64_t ws_words, uint64_t* out,
                   lgcn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Tuning (ABI 7). The schedule choices earlier builds read from environment variables at every
 * dispatch (A/B knobs) are one process-wide struct now; the library reads no environment.
 * Every default is the measured choice, so a caller that never calls lgcn_set_tuning gets the
 * tuned library. lgcn_set_tuning validates the whole struct (LGCN_E_ARG on any field out of
 * range, nothing changed) and replaces it; call it before issuing work, not concurrently with
 * calls that launch kernels. None of the fields changes a result's bits except where noted
 * (partition_*: a different, equally valid partition).
 */
typedef struct {
    /* item-pass predicated tail (a row's last < 8 edges per batch gathered together):
     * -1 = per-launch default (on for d <= 64 and for plain launches of <= 65,536 items), 0 off, 1 on */
    int32_t spmm_tail;
    /* index load rounds (batches of col/val per load round): 0 = per-width default, else one of
     * 1, 2, 4, 8, 16, 32 (widths without that instance keep their default) */
    int32_t spmm_index_rounds;
    /* lgcn_spmm_pair: XCDs (of 8) whose workgroup slots run pass a; 0 = a's blocks then b's */
    int32_t pair_xcds_a;
    /* host partitioner (lgcn_partition_*): label-propagation refinement rounds, clustering rounds */
    int32_t partition_refine_rounds;
    int32_t partition_cluster_rounds;
    /* lgcn_legacy_choice: host threads replaying the shuffles (1..256) */
    int32_t choice_threads;
    int32_t reserved[10]; /* must be zero */
} lgcn_tuning_t;
int lgcn_tuning_defaults(lgcn_tuning_t* t);
int lgcn_set_tuning(const lgcn_tuning_t* t);
int lgcn_get_tuning(lgcn_tuning_t* t);

/* ---------------------------------------------------------------------------------------
 * CSR construction. Stable counting sort of the edge list by `key`:
 *   rowptr[N+1] (int64), col[E] = other[perm] (int32), eid[E] = perm (int32),
 * where perm lists edge positions grouped by key and, inside a key, in input order.
 * Forward plan: key = edge_index[1] (target), other = edge_index[0] (source) — the
 * per-target order in which PyG's scatter(reduce='sum') adds messages on CPU.
 * Transposed plan (backward, reference Q3: train/val/test edge sets are asymmetric):
 * key = edge_index[0], other = edge_index[1] — the order of index_add_ in
 * index_select's backward.
 * Out-of-range ids (<0 or >=N) set *err_count (device int64, caller-zeroed) > 0.
 * Replaces: gcn_norm's degree scatter and scatter_add_'s implicit ordering inside
 * LGConv.forward (PyG 2.4.0 nn/conv/lg_conv.py, nn/conv/gcn_conv.py::gcn_norm),
 * called from reference models/light_gcn.py:33. */
int lgcn_csr_workspace_size(int64_t E, int64_t N, size_t* bytes);
int lgcn_csr_build(const int64_t* key, const int64_t* other, int64_t E, int64_t N,
                   int64_t* rowptr, int32_t* col, int32_t* eid, int64_t* err_count,
                   void* ws, size_t ws_bytes, lgcn_stream_t stream);

/* Key grouping without a radix sort: rowptr[R+1] and perm[B] exactly as lgcn_csr_build(key, key,
 * B, R, ...) writes rowptr and eid (positions b grouped by key[b], ascending b inside a key; an
 * out-of-range key counts in *err_count and is grouped under key 0, as there). A counting sort:
 * one atomic count per key, one scan, atomic placement, then each key's few positions put in
 * ascending order. cursor: device int32[lgcn_group_keys_cursor_len(R)] scratch whose first R
 * entries are zero on entry (allocate it zeroed) and are left zero on exit — no memset, so the
 * call captures into a hipGraph as kernels only (the tail holds per-tile totals).
 * Integrity: the kernels check every index they write through (the counts must add up to B,
 * placements and groups must lie inside perm[0, B)); a failed check adds 2^32 to *err_count and
 * drops the write instead of faulting — so *err_count >= 2^32 means the grouping is invalid
 * (below 2^32 it counts out-of-range keys). Meant for many keys over a small range with
 * short groups (the per-step negatives, B ~ 1.8e5 over I = 59,047 items: ~3 per key); a group's
 * ordering is quadratic in its length. B < 2^31, R < 2^31.
 * Replaces: the per-step grouping that index_put_(accumulate) performs implicitly in the
 * backward of compute_embeddings' negative-row gather (reference utils/train_test.py:128-132,
 * negatives from utils/helpers.py:64-82). */
int lgcn_group_keys(const int64_t* key, int64_t B, int64_t R, int64_t* rowptr, int32_t* perm, int32_t* cursor,
                    int64_t* err_count, lgcn_stream_t stream);
int64_t lgcn_group_keys_cursor_len(int64_t R);

/* gcn_norm(add_self_loops=False), PyG 2.4.0: deg = in-degree (count of edges whose target
 * is the node), dis = deg^-1/2 with inf -> 0 (computed as 1/sqrt(deg), correctly rounded
 * twice, which is what torch's CPU pow(-0.5) yields), and edge weight
 * w = dis[source] * 1 * dis[target].
 *   lgcn_inv_sqrt_degree: dis[i] from the FORWARD plan's rowptr (rows = targets).
 *   lgcn_edge_norm: val[p] = dis[row(p)] * dis[col[p]] for every slot p of any plan
 *   (forward or transposed; the product is symmetric). */
int lgcn_inv_sqrt_degree(const int64_t* rowptr_fwd, int64_t N, float* dis, lgcn_stream_t stream);
int lgcn_edge_norm(const int64_t* rowptr, const int32_t* col, int64_t N, int64_t E,
                   const float* dis, float* val, lgcn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Load-balanced schedule for one plan. Rows longer than `chunk` edges are cut into chunks
 * of `chunk` edges. Items of rows [0, side_split) come first, then the others (LightGCN passes
 * side_split = num_users, so the rows gathering from the item table run together and then the
 * rows gathering from the user table: each phase has one table's working set in L2); inside a
 * side items are ordered longest-first (stable), so neighbouring lane groups of a wave carry
 * equal work. side_split = 0 gives one global longest-first order. row_mask (device uint8[N],
 * nullable) restricts the schedule to rows with row_mask[r] != 0: rows outside it get no item, so
 * lgcn_spmm leaves them untouched (the sparse Cluster-GCN batch step schedules only the rows its
 * edges touch). Capacities: items <= N + E/chunk, splits <= N,
 * partials <= E/chunk + N. counts[0..2] (device int64) receive n_items, n_splits,
 * n_partials; the caller reads them back once per plan. */
int lgcn_schedule_workspace_size(int64_t E, int64_t N, int32_t chunk, size_t* bytes);
int lgcn_schedule_build(const int64_t* rowptr, int64_t N, int64_t E, int32_t chunk,
                        int64_t side_split, const uint8_t* row_mask, lgcn_item_t* items, int64_t items_cap,
                        lgcn_split_t* splits, int64_t splits_cap,
                        int64_t* counts, void* ws, size_t ws_bytes, lgcn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * One propagation layer out = Â x with a fused LightGCN epilogue (see LGCN_EPI_*).
 * Replaces LGConv.forward → propagate → message (w * x_j) → SumAggregation
 * (PyG 2.4.0), reference models/light_gcn.py:33, and the layer-stack mean at :36 (folded
 * into the epilogue), and — over the transposed plan — the autograd backward of both.
 * x: split table (gather source). e: split table (epilogue addend; may be NULL unless the
 * mode reads it). acc: split table (accumulator / final output). y: optional [N,d] layer
 * output (input of the next layer). partial: [n_partials, d] scratch.
 * Every row of an unmasked plan has at least one item (zero-length for zero in-degree), so the
 * epilogue covers all N rows; a row_mask plan writes only its rows. */
int lgcn_spmm(const lgcn_item_t* items, int64_t n_items,
              const lgcn_split_t* splits, int64_t n_splits,
              const int32_t* col, const float* val, int64_t N, int32_t d,
              const float* x_lo, const float* x_hi, int64_t x_split,
              const float* e_lo, const float* e_hi, int64_t e_split,
              float* y,
              float* acc_lo, float* acc_hi, int64_t acc_split,
              float* partial, int32_t mode, float div, float mul,
              lgcn_stream_t stream);

/* The two halves of lgcn_spmm, same arguments: the item pass (every unsplit row's epilogue and
 * every chunk partial) and the combine pass (split rows). lgcn_spmm == items then combine.
 * Exposed so a profiler can bracket the dominant kernel alone. */
int lgcn_spmm_items(const lgcn_item_t* items, int64_t n_items,
                    const lgcn_split_t* splits, int64_t n_splits,
                    const int32_t* col, const float* val, int64_t N, int32_t d,
                    const float* x_lo, const float* x_hi, int64_t x_split,
                    const float* e_lo, const float* e_hi, int64_t e_split,
                    float* y,
                    float* acc_lo, float* acc_hi, int64_t acc_split,
                    float* partial, int32_t mode, float div, float mul,
                    lgcn_stream_t stream);
int lgcn_spmm_combine(const lgcn_item_t* items, int64_t n_items,
                      const lgcn_split_t* splits, int64_t n_splits,
                      const int32_t* col, const float* val, int64_t N, int32_t d,
                      const float* x_lo, const float* x_hi, int64_t x_split,
                      const float* e_lo, const float* e_hi, int64_t e_split,
                      float* y,
                      float* acc_lo, float* acc_hi, int64_t acc_split,
                      float* partial, int32_t mode, float div, float mul,
                      lgcn_stream_t stream);
/* to_undirected + coalesce (reference data/dataset_handler.py:141, PyG 2.4.0 semantics): the
 * 2P keys row*N+col of both directions of the P pairs, sorted ascending and deduplicated into
 * (out_row, out_col)[*out_count] (capacity 2P). Ids outside [0, N) are counted in *err_count
 * (and clamped; the caller raises). */
int lgcn_coalesce_workspace_size(int64_t P, int64_t N, size_t* bytes);
int lgcn_coalesce_undirected(const int64_t* src, const int64_t* dst, int64_t P, int64_t N, int64_t* out_row,
                             int64_t* out_col, int64_t* out_count, int64_t* err_count, void* ws, size_t ws_bytes,
                             lgcn_stream_t stream);

/* Source-sliced schedule (lgcn_amd/sliced.py): S slices of the source id range, bounds[0..S]
 * (device int64, bounds[0] = 0, bounds[S] = N, S <= 250). Every row's CSR run is cut where its
 * neighbour's slice changes; a row with a segment longer than chunk is a hub (its segments are
 * chunked into partial slots, finished by lgcn_spmm_combine via splits), any other row gets one
 * item per segment with FIRST/LAST flags (an empty row one flag-only item in slice 0). Items are
 * sorted slice-major, longest first; offsets[s] (device int64[S+1]) is slice s's first item.
 * counts = {n_items, n_splits, n_partials, unsorted}: unsorted != 0 if some row's neighbours are
 * not ascending (the chain could not follow CSR order; use the plain schedule).
 * row_mask (device uint8[N], nullable): only rows with a nonzero mask get items (a rank's owned
 * destination rows of a row-sharded plan, lgcn_amd/sharded.py); NULL = every row. */
int lgcn_slice_schedule_workspace_size(int64_t E, int64_t N, int32_t S, int32_t chunk, size_t* bytes,
                                       int64_t* items_cap);
int lgcn_slice_schedule_build(const int64_t* rowptr, const int32_t* col, int64_t N, int64_t E,
                              const int64_t* bounds, int32_t S, int32_t chunk, const uint8_t* row_mask,
                              lgcn_item_t* items, int64_t items_cap,
                              int64_t* offsets, lgcn_split_t* splits, int64_t splits_cap, int64_t* counts,
                              void* ws, size_t ws_bytes, lgcn_stream_t stream);

/* One launch of a source-sliced schedule (the item pass only). Row items carry flags in the high
 * bits of len: 0x20000000 = the row's FIRST segment (its sum starts at 0, else it continues from
 * run[row]), 0x40000000 = its LAST segment (the epilogue runs, else the running sum is stored to
 * run[row], [N, d]); the low 29 bits are the length. Partial-slot items (dst < 0) carry no flags.
 * Issued once per slice in ascending source order, each row's sum stays one sequential chain in
 * CSR order; lgcn_spmm_combine afterwards finishes the chunked (hub) rows. */
int lgcn_spmm_run(const lgcn_item_t* items, int64_t n_items, const lgcn_split_t* splits, int64_t n_splits,
                  const int32_t* col, const float* val, int64_t N, int32_t d, const float* x_lo, const float* x_hi,
                  int64_t x_split, const float* e_lo, const float* e_hi, int64_t e_split, float* y, float* acc_lo,
                  float* acc_hi, int64_t acc_split, float* partial, int32_t mode, float div, float mul,
                  lgcn_stream_t stream, float* run);

/* All S slice launches of one layer of a source-sliced schedule in one call (the loop over
 * lgcn_spmm_run, issued from C so a layer costs one host call): slice sl is items
 * [slice_offsets[sl], slice_offsets[sl+1]) of `items`; slice_offsets is HOST memory (int64[S+1]).
 * Hub chunks (dst < 0) write their partial slots of `partial`; lgcn_spmm_combine over the hub rows
 * finishes them afterwards, as after lgcn_spmm_run. Same reference code as lgcn_spmm. */
int lgcn_spmm_run_slices(const lgcn_item_t* items, const int64_t* slice_offsets, int32_t S, const int32_t* col,
                         const float* val, int64_t N, int32_t d, const float* x_lo, const float* x_hi,
                         int64_t x_split, const float* e_lo, const float* e_hi, int64_t e_split, float* y,
                         float* acc_lo, float* acc_hi, int64_t acc_split, float* partial, int32_t mode, float div,
                         float mul, lgcn_stream_t stream, float* run);

/* One launch instead of lgcn_spmm's two (item pass + combine), for schedules whose split rows
 * have few chunks (Cluster-GCN batch plans): workgroup s < n_splits sums split row s itself —
 * its pcnt chunk items chunks[pbeg .. pbeg+pcnt) (lgcn_item_t, in partial-slot order; items keep
 * the row items only) — in the same association as item pass + combine (lane group g adds chunks
 * g, g+G, ... then the G group sums in order), so the result is bitwise lgcn_spmm's; `partial`
 * is unused (may be NULL). Vector widths only (d in {4, 8, ..., 1024}, 16-byte aligned rows).
 * Replaces the same reference code as lgcn_spmm (models/light_gcn.py:33, LGConv.propagate). */
int lgcn_spmm_blocksplit(const lgcn_item_t* items, int64_t n_items, const lgcn_split_t* splits, int64_t n_splits,
                         const int32_t* col, const float* val, int64_t N, int32_t d, const float* x_lo,
                         const float* x_hi, int64_t x_split, const float* e_lo, const float* e_hi, int64_t e_split,
                         float* y, float* acc_lo, float* acc_hi, int64_t acc_split, float* partial, int32_t mode,
                         float div, float mul, lgcn_stream_t stream, const lgcn_item_t* chunks);

/* Two independent plain passes of one width d over N-row tables, each described by the arguments
 * lgcn_spmm takes (lgcn_pass_t below), issued together: what = 1 runs both item passes in ONE
 * launch (workgroups of a first, then b's, each in its own longest-first order), what = 2 both
 * combine passes in one launch, what = 3 both. Per row the result is bitwise what lgcn_spmm_items /
 * lgcn_spmm_combine give for each pass alone; the two passes must not write what the other reads.
 * The reduce-mode sharded forward (lgcn_amd/sharded.py) pairs a layer's user pass (users from the
 * item table) with its item-partial pass (items from the rank's users): one launch gap and one
 * drain per pair instead of two. While both passes have workgroups left, pass a takes the slots the
 * round-robin dispatch deals to XCDs 0-3 and pass b those of XCDs 4-7, so each XCD's L2 caches
 * one pass's gather table (env LGCN_PAIR_XCD=0: a's workgroups, then b's, on every XCD).
 * Vector widths only (d in {4, 8, ..., 1024}, 16-byte aligned rows).
 * Replaces, like lgcn_spmm, LGConv.forward at reference models/light_gcn.py:33 (ABI 5). */
typedef struct {
    const lgcn_item_t* items;
    int64_t n_items;
    const lgcn_split_t* splits;
    int64_t n_splits;
    const int32_t* col;
    const float* val;
    const float* x_lo;
    const float* x_hi;
    int64_t x_split;
    const float* e_lo;
    const float* e_hi;
    int64_t e_split;
    float* y;
    float* acc_lo;
    float* acc_hi;
    int64_t acc_split;
    float* partial;
    int32_t mode;
    float div;
    float mul;
    /* combine layout: -1 = every split row gets a workgroup (lgcn_spmm's combine); n >= 0 = split
     * rows [0, n) get a workgroup each, rows [n, n_splits) are combined one per lane group instead
     * — the same association, so the same bits, with a fraction of the workgroups (a rank plan has
     * thousands of 2-16-chunk split rows). Rows of <= 16 chunks (pcnt <= 16) belong after n (as
     * pack_split_rows orders them); a longer row there is still combined exactly, one running sum
     * at a time by its lane group, only slower */
    int64_t n_split_big;
} lgcn_pass_t;
int lgcn_spmm_pair(const lgcn_pass_t* a, const lgcn_pass_t* b, int64_t N, int32_t d, int32_t what,
                   lgcn_stream_t stream);

/* One plain pass described by an lgcn_pass_t (what = 1 item pass, 2 combine, 3 both): lgcn_spmm
 * with the packed combine of n_split_big — bitwise lgcn_spmm's rows. The reduce-mode forward's
 * overlapped order runs its passes one at a time through this (ABI 5). Any d lgcn_spmm takes. */
int lgcn_spmm_pass(const lgcn_pass_t* p, int64_t N, int32_t d, int32_t what, lgcn_stream_t stream);

/* lgcn_spmm_run_slices with a riding combine (ABI 5): the split rows of `ride` (an lgcn_pass_t of
 * which only splits / n_splits / n_split_big / partial / e / y / acc / mode / div / mul are used,
 * its x tables must be non-NULL) are combined by extra workgroups of slice launch `ride_slice`
 * instead of by a launch of their own (an empty ride slice: a combine launch of its own). The
 * caller guarantees that slice launch neither reads nor writes the ride's rows, its partial slots
 * or its y rows. The one-GPU K-layer forward (lgcn_amd.propagate) alternates its two slice groups
 * per layer — user-table slices (which write item rows) and item-table slices (which write user
 * rows) — so each group's split rows ride in the next group's first launch, reading partials from
 * a buffer the next layer does not write: one combine launch per forward instead of one per layer.
 * Per row the same arithmetic as lgcn_spmm_run_slices + lgcn_spmm_combine (bitwise). Vector widths
 * only (d in {4, 8, ..., 1024}, 16-byte aligned rows). Same reference code as lgcn_spmm. */
int lgcn_spmm_run_slices_ride(const lgcn_item_t* items, const int64_t* slice_offsets, int32_t S, const int32_t* col,
                              const float* val, int64_t N, int32_t d, const float* x_lo, const float* x_hi,
                              int64_t x_split, const float* e_lo, const float* e_hi, int64_t e_split, float* y,
                              float* acc_lo, float* acc_hi, int64_t acc_split, float* partial, int32_t mode,
                              float div, float mul, lgcn_stream_t stream, float* run, const lgcn_pass_t* ride,
                              int32_t ride_slice);

/* The layer-stack mean of rows whose layer outputs were kept instead of accumulated (ABI 5):
 * out[r] = ((((e[r] + y_0[r]) + y_1[r]) + ... + y_{K-1}[r]) / div) * mul for r in [0, rows) — the
 * additions and roundings of the INIT, ADD..., FINAL_ACC epilogue sequence (K == 1: FINAL_E), so
 * bitwise what they give. e, out and the K (1..8) tables ys[k] (a HOST array of device pointers)
 * are [rows, d] fp32, 16-byte aligned, d % 4 == 0. The reduce-mode forward keeps its reduced item
 * rows per layer (the next user pass reads them anyway) and runs this once on its item share
 * instead of one epilogue pass per layer over every item row (reference models/light_gcn.py:36). */
int lgcn_stack_mean_rows(const float* e, const float* const* ys, int32_t K, int64_t rows, int32_t d, float* out,
                         float div, float mul, lgcn_stream_t stream);

/* out[i] = (in[i] * mul) / div over n floats: the gradient that MulBackward (× 1/(K+1))
 * then MeanBackward (÷ (K+1)) hand to every layer output (reference models/light_gcn.py:36). */
int lgcn_scale(const float* in, float* out, int64_t n, float mul, float div, lgcn_stream_t stream);

/* Split-table copy with scale: out[r] = (x[r] / div) * mul for r in [0,N) — the K == 0
 * LightGCN forward (mean over a one-element stack). */
int lgcn_copy_scale(const float* x_lo, const float* x_hi, int64_t x_split, int64_t N, int32_t d,
                    float* out, float div, float mul, lgcn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Fused cosine-BPR loss + gradient (reference utils/train_test.py:18-64 bpr_loss over the six
 * gathers of compute_embeddings :105-134). Triplet b = (u[b], p[b], n[b]) (user id, item ids).
 * F: propagated table (split; user u at row u, item i at row U+i), W: layer-0 table (same).
 *   lgcn_bpr_fused writes, per triplet, dF rows cf[b], cf[B+b], cf[2B+b] (d loss / d F rows of
 *   u, p, n), reg-gradient rows cw[...] (d loss / d W rows) and terms[b] = softplus term,
 *   terms[B+b] = sum of squares of the three W rows. d in {16,32,64,128,256,512}.
 *   touched (device uint8[N], nullable): rows with touched[r] == 0 were not propagated (a sparse
 *   batch plan) and their F row is (W[r] / div) * mul — LightGCN's output for a row no batch edge
 *   reaches (every layer adds an exact 0).
 *   lgcn_bpr_loss: loss[0] = -(mean softplus)/10 + coeff * sum(squares)/(B*d).
 *   lgcn_segment_rows: out[r] (+)= sum of C[perm[e]] for e in [rowptr[r], rowptr[r+1]) in order —
 *   the deterministic scatter of those rows, with rowptr/perm from lgcn_csr_build over the 3B keys
 *   (u, U+p, U+n). add == 0 writes every row as (sum * mul) / div (0 where empty) — with the
 *   LightGCN backward scale this is the seed g of the backward; add != 0 only adds (sum * mul) / div
 *   to rows with contributions. */
/* cw may be NULL: the reg rows are then not materialised (lgcn_reg_rows_add and the scatters'
 * reg sources form their sums from W). */
int lgcn_bpr_fused(const float* f_lo, const float* f_hi, int64_t f_split,
                   const float* w_lo, const float* w_hi, int64_t w_split, int64_t U,
                   const int64_t* u, const int64_t* p, const int64_t* n, int64_t B, int32_t d,
                   const uint8_t* touched, float div, float mul,
                   float coeff, float* cf, float* cw, float* terms, lgcn_stream_t stream);
/* Column-sharded form (exact single-GPU training split over ranks by embedding columns, SURVEY
 * §8e's parity-preserving alternative): the rows are one rank's d of d_full columns.
 *   phase 1: sums[b*6 + k] = this rank's partial of (|u|^2, |p|^2, |n|^2, u.p, u.n, reg squares)
 *            over its columns; nothing else is written;
 *   (the caller all-reduces sums over the column groups)
 *   phase 2: reads the six full sums and writes cf / cw / terms as lgcn_bpr_fused does, for this
 *            rank's columns; the reg scale uses d_full (cw rows = coeff * 2 / (B * d_full) * W).
 * d in {8, 16, ..., 512}. Replaces the same reference code as lgcn_bpr_fused. */
int lgcn_bpr_fused_cols(const float* f_lo, const float* f_hi, int64_t f_split, const float* w_lo, const float* w_hi,
                        int64_t w_split, int64_t U, const int64_t* u, const int64_t* p, const int64_t* n, int64_t B,
                        int32_t d, int32_t d_full, const uint8_t* touched, float div, float mul, float coeff, float* sums,
                        int32_t phase, float* cf, float* cw, float* terms, lgcn_stream_t stream);
/* partial: NULL, or float[2 * LGCN_LOSS_PARTS] scratch — large batches then sum in two stages
 * (LGCN_LOSS_PARTS blocks over contiguous shares, one block over the shares): a fixed association
 * either way, so the loss is deterministic. */
#define LGCN_LOSS_PARTS 256
/* batches below this many triplets sum their loss in one block (lgcn_bpr_loss without partial
 * scratch's second stage) — the sizes lgcn_range_scatter_add_loss can fold into its launch */
#define LGCN_LOSS_FUSED_MAX_B 16384
int lgcn_bpr_loss(const float* terms, int64_t B, int32_t d, float coeff, float* loss, float* partial,
                  lgcn_stream_t stream);
/* acc[0] += (double)loss[0] * w (ABI 9): the harness's epoch loss, sum of batch loss * edges
 * (reference utils/train_test.py:101-103 accumulates loss.item() * edges in Python floats: the same
 * two double roundings), a node of each batch's captured step instead of three eager launches. */
int lgcn_loss_accumulate(const float* loss, double w, double* acc, lgcn_stream_t stream);
int lgcn_segment_rows(const int64_t* rowptr, const int32_t* perm, const float* C, int64_t N, int32_t d,
                      float* out_lo, float* out_hi, int64_t split, int32_t add, float mul, float div,
                      lgcn_stream_t stream);
/* The per-step part of that scatter for the B random negatives, in ONE launch and without a
 * sort (the users/positives part has a fixed structure per batch and goes through a
 * load-balanced plan built once, with lgcn_spmm SCALE / ADD epilogues):
 * out[key_offset + keys[b]] += (sum over b,
 * in b order, of C[b]) * mul / div for keys in [0, nrows). Workgroup w owns a key range and keeps
 * its keys in b order by an ordered block compaction; used for the per-step negatives.
 * Optional second source C2 (nullable): the same per-row sums of C2 are parked in c2buf[b_first]
 * (the launch writes c2flag[b] for every b: 1 on a row's first occurrence, else 0 — no memset
 * needed) for lgcn_flagged_rows_add to add LATER (the
 * negatives' reg-gradient rows must land after the backward). *overflow (nullable, caller-zeroed)
 * is set if a workgroup's list overflowed — parked sums would then be split; callers check it.
 * store_unless (nullable, uint8[rows]): a row with store_unless[row] == 0 is STORED (not added
 * to) — the row-lazy step leaves rows outside its touched set unwritten.
 * The second source may instead be the BPR reg-gradient rows themselves (reg_w_lo non-NULL, C2
 * NULL): every occurrence of row r contributes kreg * W[r], kreg = reg_coeff * 2 / (reg_B * d)
 * (the k_bpr_fused expression, reference utils/train_test.py:38-41), so the parked sum is the n
 * occurrences' copies added in sequence — no [B, d] reg table is read. W: the layer-0 tables
 * split at reg_w_split. */
int lgcn_range_scatter_add(const int64_t* keys, int64_t B, int64_t nrows, int64_t key_offset, const float* C,
                           int32_t d, float* out_lo, float* out_hi, int64_t split, float mul, float div,
                           const float* C2, const float* reg_w_lo, const float* reg_w_hi, int64_t reg_w_split,
                           float reg_coeff, int64_t reg_B, float* c2buf, uint8_t* c2flag, int32_t* overflow,
                           const uint8_t* store_unless, lgcn_stream_t stream);
/* lgcn_range_scatter_add plus, as one extra workgroup of the same launch, lgcn_bpr_loss's
 * single-block sum (the same block size, so the same association: bitwise its result) of
 * terms[0 .. 2 loss_B) into loss[0] (ABI 4; 1 <= loss_B < LGCN_LOSS_FUSED_MAX_B, B >= 1, nrows >= 1).
 * The step's loss launch folded into a launch it needs anyway (one launch fewer per small step). */
int lgcn_range_scatter_add_loss(const int64_t* keys, int64_t B, int64_t nrows, int64_t key_offset, const float* C,
                                int32_t d, float* out_lo, float* out_hi, int64_t split, float mul, float div,
                                const float* C2, const float* reg_w_lo, const float* reg_w_hi, int64_t reg_w_split,
                                float reg_coeff, int64_t reg_B, float* c2buf, uint8_t* c2flag, int32_t* overflow,
                                const uint8_t* store_unless, const float* terms, int64_t loss_B, int32_t loss_d,
                                float loss_coeff, float* loss, lgcn_stream_t stream);
/* The same per-row work as lgcn_range_scatter_add (flags, b-order sums, parked C2 sums, store or
 * add) for LARGE B, where every range-scatter workgroup streaming all B keys would cost O(B^2):
 * the keys arrive grouped by row in b order as rowptr[nrows+1] / perm[B] (= b) from
 * lgcn_csr_build(keys, keys, B, nrows, ...), one stable radix sort. Bitwise the range scatter's
 * result (same association) and it never overflows. Replaces, like lgcn_range_scatter_add, the
 * negatives' share of the index_put_ accumulate in the backward of reference
 * utils/train_test.py:128-134 (compute_embeddings' item_embedding gathers). */
int lgcn_sorted_scatter_add(const int64_t* rowptr, const int32_t* perm, int64_t nrows, int64_t key_offset,
                            const float* C, int32_t d, float* out_lo, float* out_hi, int64_t split, float mul,
                            float div, const float* C2, const float* reg_w_lo, const float* reg_w_hi,
                            int64_t reg_w_split, float reg_coeff, int64_t reg_B, float* c2buf, uint8_t* c2flag,
                            const uint8_t* store_unless, lgcn_stream_t stream);
/* The fixed (user, positive) reg-gradient rows of a batch: rowptr counts the contributions per
 * row (a segment plan of the 2B keys); every listed row with n > 0 gets out[r] += n copies of
 * kreg * W[r] added in sequence (kreg as in lgcn_range_scatter_add). rows (device int32[n_rows],
 * nullable): the rows to visit (NULL: rows 0 .. n_rows-1). Replaces a [2B, d] reg table and its
 * ADD pass (reference utils/train_test.py:38-41, the reg term's gradient). */
/* The grouped negatives' reg-gradient rows after the backward: for every key r in [0, nrows) with
 * n = rowptr[r+1] - rowptr[r] > 0, out[r + key_offset] += n copies of coeff * 2 / (B * d) *
 * W[r + key_offset] added in sequence — what the sorted scatter would park per row and
 * lgcn_flagged_rows_add add back, without the [B, d] parking table. (lgcn_sorted_scatter_add writes
 * the first-occurrence flags whenever c2flag is given, parking or not.) */
int lgcn_grouped_reg_add(const int64_t* rowptr, int64_t nrows, int64_t key_offset, const float* w_lo,
                         const float* w_hi, int64_t w_split, int32_t d, float coeff, int64_t B, float* out_lo,
                         float* out_hi, int64_t split, lgcn_stream_t stream);
int lgcn_reg_rows_add(const int64_t* rowptr, const int32_t* rows, int64_t n_rows, const float* w_lo, const float* w_hi,
                      int64_t w_split, int32_t d, float coeff, int64_t B, float* out_lo, float* out_hi, int64_t split,
                      lgcn_stream_t stream);
int lgcn_flagged_rows_add(const int64_t* keys, int64_t B, int64_t key_offset, const float* c2buf,
                          const uint8_t* c2flag, int32_t d, float* out_lo, float* out_hi, int64_t split,
                          lgcn_stream_t stream);

/* The reg-gradient rows of a batch step by their occurrence counts (ABI 10): row r's gradient gets
 * nf copies of kreg * W[r] (its (user, positive) occurrences, fixed_rowptr[r+1] - fixed_rowptr[r])
 * and then nn copies (its negatives': neg_rowptr[r-neg_off+1] - neg_rowptr[r-neg_off], or
 * neg_count[r - neg_off], for neg_off <= r < neg_off + neg_rows), each sum formed in sequence from 0
 * and added only when it has copies, kreg = coeff * 2 / (B * d) — exactly what lgcn_reg_rows_add
 * then lgcn_flagged_rows_add / lgcn_grouped_reg_add add after the backward (reference
 * utils/train_test.py:38-41). lgcn_row_grad_norm_reg and lgcn_row_adam_reg form them on the fly
 * (the norm from W, the update from the parameter rows before any replay — the same rows), so the
 * single-GPU step needs neither pass nor a parked sum. fixed_rowptr nullable (no fixed copies). */
typedef struct {
    const float* w_lo; /* the layer-0 tables (the parameters), split at w_split rows */
    const float* w_hi;
    int64_t w_split;
    float coeff;
    int64_t B; /* triplets in the batch (>= 1) */
    const int64_t* fixed_rowptr; /* [N + 1] or NULL */
    const int64_t* neg_rowptr;   /* [neg_rows + 1] (grouped negatives) — or ... */
    const int32_t* neg_count;    /* ... [neg_rows] (lgcn_range_scatter_add_counts); exactly one when neg_rows > 0 */
    int64_t neg_off;
    int64_t neg_rows;
} lgcn_reg_rows_t;
/* lgcn_range_scatter_add for the reg rows' counted form (ABI 10): no second source, no parked sum;
 * instead reg_count[r] (int32[nrows], every row written) = the number of keys of row r, and c2flag as
 * always. terms (nullable): with loss / loss_B / loss_d / loss_coeff, the step's loss as
 * lgcn_range_scatter_add_loss sums it; loss_acc (nullable, needs terms): then also
 * loss_acc[0] += (double)loss[0] * loss_w in the same workgroup, as lgcn_loss_accumulate adds it. */
int lgcn_range_scatter_add_counts(const int64_t* keys, int64_t B, int64_t nrows, int64_t key_offset, const float* C,
                                  int32_t d, float* out_lo, float* out_hi, int64_t split, float mul, float div,
                                  uint8_t* c2flag, int32_t* overflow, const uint8_t* store_unless, int32_t* reg_count,
                                  const float* terms, int64_t loss_B, int32_t loss_d, float loss_coeff, float* loss,
                                  double* loss_acc, double loss_w, lgcn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Row-lazy Adam (lgcn_rowadam.hip) for the sparse batch step: exact replay of the zero-gradient
 * steps a row missed, when the row is next touched (reference utils/train_test.py:95-96; same
 * element arithmetic as lgcn_adam_step). Tables p/g/m/v are (lo, hi) split at `split` rows of d.
 *   lgcn_adam_consts: consts[t] = (s, c, 1.0f / c, 0) with s = float(-lr / (1 - beta1^t)) and
 *     c = float(sqrt(1 - beta2^t)), t in [t0, t1] (4 floats per step, 16-byte aligned; ABI 6 — ABI 5
 *     had (s, c) pairs), the lgcn_adam_prologue formulas; consts[0].x = 1 when beta2 is
 *     exactly 0.999 (the schedule whose step-constant division lgcn_row_adam may take by Markstein's
 *     proven-exact shortcut; set by a call with t0 = 1, cleared by a call with another beta2), else 0.
 *   lgcn_row_adam: rows = rows_a[0..n_a) then keys_b[j] + off_b (j counted only if first_b[j]
 *     and !skip_b[row], when those are given). *step = completed steps (device int64).
 *     mode 0: catch the rows up to *step (duplicates handled by claim stamps, claim initialised
 *     to -1); mode 1: catch up, then apply step *step + 1 with the gradient times clip[1]
 *     (clip nullable), then ++*step (rows must be unique); mode 2: every row of [0, n_rows) up
 *     to *step; mode 3: as mode 1 after lgcn_row_grad_norm advanced *step already (catch up to
 *     *step - 1, apply *step, no advance launch). last[r] = the last step applied to row r.
 *   lgcn_row_grad_norm: out = (||g over the listed rows||, min(max_norm / (norm + 1e-6), 1));
 *     step_advance (nullable): ++*step_advance in the same launch (then lgcn_row_adam mode 3). */
int lgcn_adam_consts(float* consts, int64_t t0, int64_t t1, float lr, double beta1, double beta2,
                     lgcn_stream_t stream);
int lgcn_row_adam(float* p_lo, float* p_hi, float* g_lo, float* g_hi, float* m_lo, float* m_hi, float* v_lo,
                  float* v_hi, int64_t split, int32_t d, const int32_t* rows_a, int64_t n_a, const int64_t* keys_b,
                  int64_t n_b, int64_t off_b, const uint8_t* first_b, const uint8_t* skip_b, int64_t n_rows,
                  int32_t* last, int32_t* claim, int64_t* step, const float* consts, float one_minus_beta1,
                  float beta2, float one_minus_beta2, float eps, const float* clip, int32_t mode,
                  lgcn_stream_t stream);
int lgcn_row_grad_norm_workspace_floats(void);
int lgcn_row_grad_norm(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                       int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                       const uint8_t* skip_b, float max_norm, float* ws, float* out, int64_t* step_advance,
                       lgcn_stream_t stream);
/* lgcn_row_adam (mode 1 or 3) and lgcn_row_grad_norm over g + the step's reg rows (lgcn_reg_rows_t,
 * ABI 10): bitwise those calls after lgcn_reg_rows_add and the negatives' reg pass; g is not written. */
int lgcn_row_adam_reg(float* p_lo, float* p_hi, float* g_lo, float* g_hi, float* m_lo, float* m_hi, float* v_lo,
                      float* v_hi, int64_t split, int32_t d, const int32_t* rows_a, int64_t n_a, const int64_t* keys_b,
                      int64_t n_b, int64_t off_b, const uint8_t* first_b, const uint8_t* skip_b, int32_t* last,
                      int64_t* step, const float* consts, float one_minus_beta1, float beta2, float one_minus_beta2,
                      float eps, const float* clip, int32_t mode, const lgcn_reg_rows_t* reg, lgcn_stream_t stream);
int lgcn_row_grad_norm_reg(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                           int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                           const uint8_t* skip_b, float max_norm, float* ws, float* out, int64_t* step_advance,
                           const lgcn_reg_rows_t* reg, lgcn_stream_t stream);
/* The clip norm split for the owner-sharded exchange (each rank owns some rows; the norm is over
 * all ranks' rows): lgcn_row_grad_sqnorm writes the lgcn_row_grad_norm_workspace_floats() block
 * partials of the listed rows' sum of squares (fixed block assignment: deterministic for a
 * fixed list); lgcn_row_grad_norm_finish sums nparts partials (e.g. every rank's, all-gathered,
 * in rank order) and writes out / advances step_advance as lgcn_row_grad_norm does. */
int lgcn_row_grad_sqnorm(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                         int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                         const uint8_t* skip_b, float* partials, lgcn_stream_t stream);
int lgcn_row_grad_norm_finish(const float* partials, int64_t nparts, float max_norm, float* out, int64_t* step_advance,
                              lgcn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Recall@k (reference utils/train_test.py:165-212, compute_recall_at_k, called from evaluate
 * :136-163): per sampled user row, the number of positives (candidate index < P) among the
 * top-k cosine scores against all M = P + P' candidate rows, without the [Q, M] score matrix.
 *   lgcn_recall_width: D = padded width the kernels use for d (a power of two >= 8, d <= 256)
 *     and the multiple Q must be padded to.
 *   lgcn_normalize_rows: out[r, :D] = x[idx ? idx[r] : r, :d] / ||.||_2, zero-padded columns;
 *     rows in [rows, out_rows) are zero (query padding).
 *   lgcn_score_filter: f32 MFMA scores of Q queries vs candidates r*stride (r < M); thr == NULL
 *     writes every score at slot r of each query's list (dense mode, M <= cap), otherwise keys
 *     >= thr[q] are appended (list_n[q] += 1; caller zeroes list_n; overflow past cap is
 *     counted but not stored).
 *   lgcn_select_topk: per query, the k-th largest key of its list (dense_n entries when list_n
 *     is NULL) -> thr_out[q]; and/or hits_out[q] = positives ranked in the top k (ties take the
 *     lowest candidate index first), -1 if the list holds fewer than k entries.
 * Keys are order-preserving uint32 images of the f32 scores (NaN highest). */
int lgcn_recall_width(int32_t d, int32_t* D_out, int32_t* qpad_multiple);
int lgcn_normalize_rows(const float* x, const int64_t* idx, int64_t rows, int64_t ld, int32_t d, float* out,
                        int32_t D, int64_t out_rows, lgcn_stream_t stream);
int lgcn_score_filter(const float* Qn, int64_t Qpad, int64_t Qvalid, const float* Cn, int64_t M, int64_t stride,
                      int32_t D, const uint32_t* thr, uint32_t* list_key, int32_t* list_idx, int32_t* list_n,
                      int32_t cap, lgcn_stream_t stream);
int lgcn_select_topk(const uint32_t* list_key, const int32_t* list_idx, const int32_t* list_n, int32_t dense_n,
                     int32_t cap, int32_t k, int64_t P, int64_t Qpad, int64_t Qvalid, uint32_t* thr_out,
                     int32_t* hits_out, lgcn_stream_t stream);
/* CPU torch.topk's tie rule (ABI 9; replaces torch.topk(scores, k) at reference
 * utils/train_test.py:197 as the reference runs it on a CPU): hits_out[q] = positives (index < P)
 * among the k slots ATen's CPU topk fills — std::partial_sort when k * 64 <= M (k <= 4096), else
 * std::nth_element(k - 1), libstdc++'s algorithms reproduced step for step on the (key, index)
 * sequence — so the set chosen among EQUAL scores is the CPU reference's, not the lowest indices.
 * list_key/list_idx: lgcn_score_filter's dense rows (stride 1, cap >= M); both are overwritten
 * (the nth_element path permutes them in place). Padding queries [Qvalid, Qpad) get 0. */
int lgcn_select_topk_stl(uint32_t* list_key, int32_t* list_idx, int64_t cap, int64_t M, int32_t k, int64_t P,
                         int64_t Qpad, int64_t Qvalid, int32_t* hits_out, lgcn_stream_t stream);

/* Host-only (no GPU): `draws` consecutive numpy legacy np.random.choice(n, size, replace=False)
 * calls (reference utils/train_test.py:187) on the MT19937 state (key[624], *pos) of
 * np.random.get_state(), written to out[draws*size]; key/pos are advanced exactly as numpy would
 * advance them, so np.random.set_state() with them continues the caller's stream unchanged. */
int lgcn_legacy_choice(uint32_t* key, int32_t* pos, int64_t n, int64_t size, int64_t draws, int64_t* out);

/* ---------------------------------------------------------------------------------------
 * Training-step tail (reference utils/train_test.py:95-96: clip_grad_norm_(max_norm=1) then
 * optim.Adam(lr=1e-3).step() over the two dense embedding tables). Device pointers; the
 * tensor descriptors themselves are a host array of n (<= 8) entries.
 *   lgcn_grad_norm: out[0] = ||all grads||_2, out[1] = min(max_norm / (out[0] + 1e-6), 1);
 *     ws holds lgcn_grad_norm_workspace_floats() floats. Deterministic two-stage reduction.
 *   lgcn_adam_step: per element g *= clip[1] (clip may be NULL), m += (1-b1)(g-m),
 *     v = b2 v + (1-b2) g^2, p += step_size * m / (sqrt(v)/bc2_sqrt + eps), with
 *     step_size = -lr/(1-b1^t) and bc2_sqrt = sqrt(1-b2^t) computed by the caller in double
 *     (as torch does); write_grad != 0 also stores the clipped g back. */
typedef struct {
    float* param;
    float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
} lgcn_adam_tensor_t;

int lgcn_grad_norm_workspace_floats(void);
int lgcn_grad_norm(const lgcn_adam_tensor_t* tensors, int32_t n, float max_norm, float* ws, float* out,
                   lgcn_stream_t stream);
int lgcn_adam_step(const lgcn_adam_tensor_t* tensors, int32_t n, float one_minus_beta1, float beta2,
                   float one_minus_beta2, float eps, float step_size, float bc2_sqrt, const float* clip,
                   const float* dev_scalars, int32_t write_grad, lgcn_stream_t stream);
/* Capturable form: lgcn_adam_prologue advances a device step counter (double) and writes
 * scalars[0] = -lr/(1-b1^t), scalars[1] = sqrt(1-b2^t); pass scalars as dev_scalars to
 * lgcn_adam_step (its step_size / bc2_sqrt arguments are then ignored). */
int lgcn_adam_prologue(double* step, float lr, double beta1, double beta2, float* scalars, lgcn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Row-sparse gradient exchange (lgcn_exchange.hip) for data-parallel Cluster-GCN training with
 * the row-lazy Adam: replaces the dense all_reduce of both embedding gradients per step (the
 * DP form of reference utils/train_test.py:92-96) by an all_gather of each rank's
 * nonzero gradient rows.
 *   lgcn_rows_pack: slot i < n_a + n_b holds the listed row (rows_a, then keys_b[j] + off_b,
 *     filtered by first_b / skip_b as in lgcn_row_adam) -> ids[i] and rows[i, :] = g[row];
 *     filtered and trailing slots (up to cap) get ids[i] = -1.
 *   lgcn_rows_mark_first: first[i] = 1 iff ids[i] >= 0 is the lowest index holding that row;
 *     claim int32[N] must hold INT32_MAX on entry and holds it again on exit.
 *   lgcn_rows_accumulate: for r = 0..world-1 in order, over slots [r*cap, (r+1)*cap):
 *     g[row] = first ? rows[i] : g[row] + rows[i]; then, if div > 0, g[row] /= div once per row.
 *     Rank r's rows start at rows + r*rank_stride (floats; >= cap*d, a multiple of 4): cap*d for
 *     separate row tables, cap*(d+2) for the one-collective records [ids as 2*cap floats | rows]. */
int lgcn_rows_pack(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                   int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                   const uint8_t* skip_b, int64_t cap, int64_t* ids, float* rows, lgcn_stream_t stream);
int lgcn_rows_mark_first(const int64_t* ids, int64_t n, int32_t* claim, uint8_t* first, lgcn_stream_t stream);
int lgcn_rows_accumulate(const int64_t* ids, const float* rows, int64_t world, int64_t cap, int64_t rank_stride,
                         const uint8_t* first, float* g_lo, float* g_hi, int64_t split, int32_t d, float div,
                         lgcn_stream_t stream);

/* Owner-sharded exchange (lgcn_amd.owner.OwnerExchange; the all_gather above replaced by two
 * all_to_alls): row r is owned by rank r % world, which alone holds its Adam state and applies its
 * update; each rank sends its gradient rows to their owners and asks the owners for the rows its
 * next step reads. A send buffer is world destination blocks of block_floats floats:
 *   [gradient ids: 2*cap floats (int64, -1 = empty) | gradient rows: cap*d | pad |
 *    request ids at float offset req_off: 2*rcap floats (int64, -1 = empty) | pad]
 *   lgcn_owner_reset: every id slot := -1, counts[0 .. 2*world) := 0.
 *   lgcn_owner_pack_rows: each listed gradient row (the lgcn_row_adam list, first_b / skip_b
 *     filters) into destination row % world at the next free slot (counts[o]); a full
 *     destination sets *overflow |= 1 (the row is dropped: the caller must check).
 *   lgcn_owner_pack_requests: each listed row id (rows_a, then keys_b + off_b; duplicates allowed)
 *     into destination row % world's request slots (counts[world + o]) and mine[o*rcap + slot];
 *     full: *overflow |= 2. claim (nullable, int32[N]; ABI 8): each distinct row requested once —
 *     stamp (>= 0) must differ from every value claim held before the call (callers keep claim at
 *     -1 initially and pass an increasing stamp), so a destination needs at most its share of
 *     the distinct rows (a structured graph's large batches draw each item many times).
 *   lgcn_rows_gather: rows[i] = p[ids[i]] for ids[i] >= 0 (scatter != 0: p[ids[i]] = rows[i]).
 *   lgcn_rows_mark: mask[ids[i]] = value for ids[i] >= 0 (and first[i], if first is given).
 * Replaces the same reference step as lgcn_rows_pack (utils/train_test.py:92-96 under DP). */
int lgcn_owner_reset(float* send, int64_t world, int64_t block_floats, int64_t cap, int64_t req_off, int64_t rcap,
                     int32_t* counts, lgcn_stream_t stream);
int lgcn_owner_pack_rows(const float* g_lo, const float* g_hi, int64_t split, int32_t d, const int32_t* rows_a,
                         int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b, const uint8_t* first_b,
                         const uint8_t* skip_b, int64_t world, int64_t cap, int64_t block_floats, int32_t* counts,
                         float* send, int32_t* overflow, lgcn_stream_t stream);
int lgcn_owner_pack_requests(const int32_t* rows_a, int64_t n_a, const int64_t* keys_b, int64_t n_b, int64_t off_b,
                             int64_t world, int64_t rcap, int64_t block_floats, int64_t req_off, int32_t* counts,
                             float* send, int64_t* mine, int32_t* overflow, int32_t* claim, int32_t stamp,
                             lgcn_stream_t stream);
int lgcn_rows_gather(const float* p_lo, const float* p_hi, int64_t split, int32_t d, const int64_t* ids, int64_t n,
                     float* rows, int32_t scatter, lgcn_stream_t stream);
int lgcn_rows_mark(const int64_t* ids, const uint8_t* first, int64_t n, uint8_t* mask, int32_t value,
                   lgcn_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Launch programs (ABI 11): a captured hipGraph issued as plain launches on a stream.
 * The fused Cluster-GCN step (reference utils/train_test.py:86-101, one batch) is captured once
 * per batch; hipGraphLaunch costs the GPU ~8 us of its own per replay, the same kernels launched
 * on the stream run back to back. lgcn_program_from_graph reads a graph's nodes once (kernels:
 * function, grid, block, dynamic LDS and the node's own argument buffers; memsets; empty nodes
 * dropped) in a dependency order (ready nodes lowest index first, so a one-stream
 * capture keeps its order); lgcn_program_run issues them on `stream` in that order, from one call,
 * no sync. The graph (hipGraph_t) must outlive the program: its nodes own the argument buffers.
 * A graph holding copy, event, host or child-graph nodes, or a kernel launched with `extra`
 * arguments, is refused with LGCN_E_UNSUPPORTED (the caller keeps replaying the graph). Host calls. */
int lgcn_program_from_graph(void* graph, void** prog_out);
int lgcn_program_launches(const void* prog);  /* kernels + memsets it issues per run */
int lgcn_program_run(const void* prog, lgcn_stream_t stream);
int lgcn_program_free(void* prog);

/* ---------------------------------------------------------------------------------------
 * Host-side (no GPU): balanced k-way node partition for Cluster-GCN batching, the METIS
 * replacement for PyG ClusterData (reference data/dataset_handler.py:273). Deterministic
 * restreaming Linear Deterministic Greedy over the undirected adjacency of (src[e], dst[e]) —
 * of the nodes, and of size-constrained label-propagation clusters (the better result kept);
 * part_out[N] receives ids in [0, num_parts); `imbalance` is the streaming capacity slack and a
 * final fix-up leaves every part with exactly floor or ceil(N/num_parts) nodes. Host pointers. Errors: lgcn_partition_last_error(). */
int lgcn_partition_edges(const int64_t* src, const int64_t* dst, int64_t E, int64_t N,
                         int32_t num_parts, int32_t passes, float imbalance, int32_t* part_out);
const char* lgcn_partition_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* LGCN_H */
