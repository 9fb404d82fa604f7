/*
 * leakgnn.h — C ABI of the MI355X-native GNN message-passing library (libleakgnn.so).
 *
 * This is the drop-in boundary for the hot path of Mateng0228/Leak-det-gnn:
 * the GCN message passing inside models/detector.py::LeakDetector (forward and
 * backward).  The reference has no FFI of its own: its hot path calls PyG
 * (`torch_geometric.nn.GCNConv`, `global_mean_pool`; detector.py:23,162-164,199,215)
 * and plain torch indexing.  Each entry point below names the reference call it
 * replaces (file:line relative to the reference repository root).  The Python
 * binding a maintainer would add on the reference side is shown in INTEGRATION.md.
 *
 * Conventions (all entry points):
 *  - Pointers are DEVICE pointers (caller-owned, e.g. PyTorch caching allocator)
 *    unless the parameter name ends in `_host`.  The library never allocates:
 *    callers pass workspace sized by the matching *_workspace_bytes() query.
 *  - Work is enqueued on `stream` (a hipStream_t; NULL = legacy default stream).
 *    No entry point synchronises the device or the host, so every call is
 *    capturable into a hipGraph.
 *  - Return value: LG_OK (0) or a negative LG_E* code; lg_strerror() names it.
 *    A launch failure returns LG_EHIP.  Compute entry points keep no mutable global
 *    state and are reentrant.  Two OPTIONAL facilities hold state, both documented
 *    at their declarations: the reduce batch (per host thread: begin and flush must
 *    come from the same thread; a flush on another thread returns LG_EINVAL and the
 *    batch stays open on its own thread) and the kernel-timing slots (one process-wide
 *    set of event pairs plus a per-thread armed slot; measurement only).  A caller that
 *    uses neither sees a stateless library.
 *  - Node features are fp32, row-major [B][N][D] (window-major, then node, then
 *    feature; one 4·D-byte row per node).  B identical graphs form the disjoint
 *    union of reference detector.py:105-114; the library keeps ONE single-graph
 *    CSR and offsets rows by b·N itself, so the (2, B·E) batchified edge_index is
 *    never materialised on the hot path.
 *  - Supported feature widths D: 32, 64 (LG_EUNSUPPORTED otherwise).
 *  - Row indices (b·N + n, b·P + p) are 32-bit inside the kernels: B·N and B·P must
 *    be < 2^31 (LG_EUNSUPPORTED otherwise).  Feature tensors larger than 4 GiB are
 *    fine: the GCN entry points split the launch over windows internally.
 */
#ifndef LEAKGNN_H
#define LEAKGNN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* lg_stream_t; /* hipStream_t */

enum {
    LG_OK = 0,
    LG_EINVAL = -1,        /* bad argument (null pointer, negative size, index out of range) */
    LG_EUNSUPPORTED = -2,  /* unsupported feature width / flag combination */
    LG_EHIP = -3           /* HIP launch or runtime error */
};

/* flags for lg_gcn_fwd / lg_gcn_bwd */
#define LG_F_BIAS      0x01  /* fwd: add bias                                                  */
#define LG_F_RELU      0x02  /* fwd: ReLU after bias (F.relu, detector.py:200)                 */
#define LG_F_DROPOUT   0x04  /* fwd: inverted dropout after ReLU (nn.Dropout, detector.py:201) */
#define LG_F_MASK_IN   0x08  /* bwd: dz = dy * scale_in * [y > 0]  (ReLU/dropout backward of THIS layer's output) */
#define LG_F_MASK_OUT  0x10  /* bwd: dx_out = dx * scale_out * [x > 0] (ReLU/dropout backward of the PREVIOUS op) */
/* bwd with node_slot / dnode_bias (ABI 20): rows of dx_out whose node has no sensor
 * (node_slot[n] < 0) MAY be left unwritten; their masked sums are in dnode_bias.  The node
 * init's backward (lg_sensor_proj_bwd) reads only the sensor rows (detector.py:181-186), so
 * layer 0's backward then writes 29 of L-TOWN-A's 661 rows per window instead of all of
 * them.  Honoured by the default node-major schedule of lg_gcn_bwd_nm[_bits]; the other
 * schedules and lg_gcn_bwd write every row. */
#define LG_F_DX_SENSOR_ROWS 0x10000000
/* Node-feature layout for lg_node_init_fwd / lg_pipe_scatter_bwd / lg_edge_head_* /
 * lg_pool_head_fwd: without it node rows are window-major [B][N][D] (row b*N + n, the
 * reference's disjoint-union order, detector.py:105-114, 192-196); with it they are
 * node-major [N][B][D] (row n*B + b), the layout of lg_gcn_fwd_nm / lg_gcn_bwd_nm.
 * Dropout masks are indexed by the window-major row in both layouts. */
#define LG_F_NODE_MAJOR 0x20
/* The bf16 node-MLP tier (BASELINE configs[2], SURVEY §8 d C3: "bf16 for K2/K5/K9 GEMMs
 * with fp32 accumulate"): lg_gcn_fwd_nm / lg_gcn_bwd_nm / lg_edge_head_fwd /
 * lg_edge_head_bwd run their products as ONE bf16 MFMA (operands rounded to bf16, fp32
 * accumulate, fp32 in HBM) instead of the 3-way split that holds fp32 accuracy.  Not an
 * fp32-parity mode: its bar is 2e-2 relative on logits against the fp32 oracle (SURVEY
 * §7).  Ignored by the kernels that have no bf16 form (they compute fp32). */
#define LG_F_BF16 0x40
/* Dropout seeds: every forward entry point taking (seed, salt) reads `seed` as the address
 * of a device-resident uint64 when salt has bit 31 set (the salt proper is bits 0..30).  A
 * captured HIP graph of a training step then re-draws its dropout streams on each replay by
 * refreshing that word on the device, with no host involvement. */
#define LG_SALT_SEED_PTR 0x80000000u
/* lg_gcn_fwd_nm[_bits] kernel and transform.  No bit: the fp32 tier runs the producer /
 * consumer pipeline (k_gcn_fwd_pc: gather waves hand (A x) tiles to MFMA waves through an LDS
 * ring) with the transform as a 2-way fp16 split with power-of-two block scaling (3 f16 MFMAs
 * per product; fp32-level accuracy, ~4e-7 of max |y|); the bf16 tier (LG_F_BF16) the per-wave
 * pipeline k_gcn_fwd_nm3 with ONE bf16 product.
 *   LG_F_BF16X3: the pc pipeline with the 3-way bf16 split (6 bf16 MFMAs per product, ~1e-8 of
 *                max |y|; bit-identical to LG_F_NM3);
 *   LG_F_NM3:    the per-wave pipeline with the 3-way bf16 split;
 *   LG_F_F32_MFMA: the per-wave pipeline on exact v_mfma_f32_16x16x4_f32 (bit-identical to
 *                lg_gcn_fwd on the transposed layout);
 *   LG_F_PC:     with LG_F_BF16: the pc pipeline's single bf16 product. */
#define LG_F_F32_MFMA      0x00400000
#define LG_F_PC            0x00004000
#define LG_F_BF16X3        0x00008000
#define LG_F_NM3           0x00020000

int lg_abi_version(void);

/* Reduce batch (ABI 12).  The backward entry points end in a deterministic slab reduction
 * of their weight/bias gradients (lg_gcn_bwd[_nm], lg_sensor_proj_bwd, lg_edge_head_bwd,
 * lg_pool_head_bwd, lg_gru_bwd, lg_linear_dw).  Between lg_reduce_batch_begin() and
 * lg_reduce_batch_flush(stream) on the SAME host thread those reductions are recorded
 * instead of launched, and the flush launches them together (one launch per 16
 * segments); every gradient column is summed in the same order, so results are unchanged.
 * Until the flush is enqueued the recorded outputs are undefined and the recorded
 * workspaces must stay allocated and unwritten.  A lg_sensor_proj_bwd whose dbias_in is
 * a recorded output folds that output's partials into its own db reduction.  Replaces
 * nothing in the reference: it merges the per-op launches of one backward pass
 * (the autograd of detector.py:170-218).  begin: LG_EINVAL when a batch is already open;
 * flush: LG_EINVAL when none is.  The open batch is THREAD-LOCAL state: a flush from a
 * thread that did not begin it returns LG_EINVAL (nothing launched, the other thread's
 * batch untouched), and a thread that exits with an open batch drops its records. */
int lg_reduce_batch_begin(void);
int lg_reduce_batch_flush(lg_stream_t stream);

/* Measurement helper (bench.py's stream_copy, the achievable-HBM reference beside the
 * 8 TB/s roofline): dst = src over `bytes` (a multiple of 16) with 16-byte non-temporal
 * loads and stores.  No reference counterpart. */
int lg_stream_copy(const void* src, void* dst, int64_t bytes, lg_stream_t stream);

/* Device dropout-seed slots (the seeds LG_SALT_SEED_PTR call sites read at launch): *state
 * += 1, then slots[i] = splitmix64(*state * n + i + 1) & (2^62 - 1), i < n <= 4096, in ONE
 * single-wave launch on the device, so a captured training step re-draws its dropout
 * streams at every replay without the host.  No reference counterpart (the reference's
 * nn.Dropout draws from torch's generator). */
int lg_seed_slots_advance(uint64_t* slots, int64_t n, uint64_t* state, lg_stream_t stream);

/* Replay of a captured step: hipGraphLaunch(graph_exec, stream), n times in a row (graph_exec:
 * an instantiated hipGraphExec_t, e.g. torch.cuda.CUDAGraph.raw_cuda_graph_exec()).  Replaces
 * nothing in the reference (its training step is eager, train_detector.py:296-317). */
int lg_graph_replay(void* graph_exec, int64_t n, lg_stream_t stream);
const char* lg_strerror(int code);

/* Training loss: nn.CrossEntropyLoss() (mean over rows whose target != ignore_index;
 * reference train_detector.py:235, 311) over logits [B][C] (row stride ldx).
 *   fwd: loss (device fp32 scalar), lse [B] (saved for the backward), rowloss [B] scratch;
 *        ONE launch (ABI 23): the rows, and the workgroup that finishes last forms the mean
 *        over rows in row order.  counter: a device uint32, 0 between launches (the launch
 *        resets it); one per stream that may run this concurrently.
 *   bwd: dlogits[b][c] = grad_loss[0] / n * (exp(x - lse[b]) - [c == target[b]]), 0 for
 *        ignored rows (row stride ldd).  Three launches for what torch runs as six. */
int lg_cross_entropy_fwd(const float* logits, const int64_t* target, int64_t B, int64_t C, int64_t ldx,
                         int64_t ignore_index, float* loss, float* lse, float* rowloss, unsigned* counter,
                         lg_stream_t stream);
int lg_cross_entropy_bwd(const float* logits, const int64_t* target, const float* lse, const float* grad_loss,
                         int64_t B, int64_t C, int64_t ldx, int64_t ignore_index, float* dlogits, int64_t ldd,
                         lg_stream_t stream);

/* Training-step tail: torch.nn.utils.clip_grad_norm_(params, max_norm) then
 * torch.optim.AdamW.step() (reference train_detector.py:313-317), ONE launch (ABI 23; two
 * before), two when the parameters need more 1024-element slices than the device has CUs.
 *   table : int64 [T][4] (HOST array) device addresses of (param, grad, exp_avg, exp_avg_sq), fp32
 *   sizes : int64 [T] (HOST array) element counts, T <= 48 (passed by value to the launches, so
 *           captured launches need no host copy)
 *   step  : device fp32 [4] (ABI 25; [2] before): step[0] the AdamW step counter (incremented);
 *           step[1] the launch's workgroup arrival / ticket counter, read as uint32, which must
 *           be 0 between launches (zeros at creation; the launch resets it); step[2] an error
 *           word (uint32, sticky): nonzero when a grid-barrier wait timed out, results invalid;
 *           step[3] reserved
 *   max_norm <= 0: no clipping.  norm_out (device fp32, may be NULL): the pre-clip total norm.
 *   workspace: lg_clip_adamw_workspace_bytes(sizes, T) bytes (ABI 25: one fp64 partial sum of
 *           squares per slice; each workgroup reads and writes only its own gradient slice).
 * The norm is summed in fp64 in a fixed order (deterministic; the one- and two-launch forms
 * give identical bits). */
int64_t lg_clip_adamw_workspace_bytes(const int64_t* sizes, int T);
int lg_clip_adamw(const int64_t* table, const int64_t* sizes, int T, float* step, float lr, float beta1,
                  float beta2, float eps, float weight_decay, float max_norm, float* norm_out, void* workspace, int64_t ws_bytes,
                  lg_stream_t stream);
/* lg_clip_adamw, then (ABI 23) the draw of lg_seed_slots_advance(seed_slots, n_slots, seed_state)
 * in the same launch, by its last workgroup: a captured training step ends by drawing the NEXT
 * replay's dropout seeds, one launch fewer per step. */
int lg_clip_adamw_seeds(const int64_t* table, const int64_t* sizes, int T, float* step, float lr, float beta1,
                        float beta2, float eps, float weight_decay, float max_norm, float* norm_out, void* workspace,
                        int64_t ws_bytes, uint64_t* seed_slots, int64_t n_slots, uint64_t* seed_state,
                        lg_stream_t stream);

/* Hand-off error word (ABI 25; no reference counterpart).  The producer / consumer trunk
 * forward (k_gcn_fwd_pc) bounds every LDS hand-off poll; a poll that runs out sets a bit of a
 * device word (1: producer / W staging, 2: consumer), and that launch's results are invalid.
 * lg_spin_errors copies the word to *out (synchronous, device-wide) and zeroes it if reset. */
int lg_spin_errors(uint32_t* out, int reset);

/* Kernel timing (bench.py; no reference counterpart — the reference has no kernels).
 * lg_timing_arm(slot): the NEXT library kernel launch on this host thread that is the main
 * kernel of an entry point (lg_gcn_fwd[_nm], lg_gcn_bwd[_nm], lg_edge_head_fwd/bwd,
 * lg_gru_fwd/bwd, lg_node_init_fwd, lg_pipe_scatter, lg_pool_head_fwd/bwd, lg_linear_dw,
 * lg_spmm) is launched with hipExtLaunchKernelGGL and the event pair of `slot` (created on
 * first use, reused after; process-wide, so a call on another thread, e.g. autograd's
 * worker, is read back on the caller's): their elapsed time is that kernel's own execution, as a
 * profiler's kernel trace reports it.  lg_timing_disarm returns 1 if the armed pair was
 * never consumed (and drops it), else 0.  lg_timing_elapsed: milliseconds of `slot` once
 * its stop event has completed.  Not for use inside stream capture. */
int lg_timing_arm(int slot);
int lg_timing_disarm(void);
int lg_timing_elapsed(int slot, float* ms);

/* ---------------------------------------------------------------------------
 * K4  gcn_norm + CSR build, once per graph.
 * Replaces: PyG GCNConv.forward -> gcn_norm (add_remaining_self_loops, degree,
 * deg^-1/2, w = dis[src]*dis[dst]) recomputed on every call because the
 * reference constructs GCNConv with cached=False (detector.py:163, 199).
 * Semantics (PyG published algorithm):
 *   add_self_loops: drop existing (i,i) edges, then append (i,i) for every node
 *                   with weight fill_value (1.0; 2.0 for improved=True)
 *   normalize:      deg[d] = sum of weights of edges into d;  dis = deg^-1/2 (inf -> 0);
 *                   w_e = dis[src] * weight_e * dis[dst].     normalize=0 -> w_e = weight_e.
 * Output CSR is keyed by destination (rowptr/col/w) and its transpose keyed by
 * source (rowptr_t/col_t/w_t, used by the backward pass).  Inside each row the
 * entries keep ascending edge order, appended self loop last — the order PyG's
 * scatter_add visits them — so rowptr/col are bit-exact and deterministic.
 *   edge_index : int64 [2][E] device (row 0 = source, row 1 = target)
 *   rowptr, rowptr_t : int32 [N+1];  col, col_t : int32 [E+N];  w, w_t : fp32 [E+N]
 *   rowptr[N] receives the entry count (E minus dropped loops, plus N loops).
 * ------------------------------------------------------------------------- */
int64_t lg_graph_workspace_bytes(int64_t E, int64_t N);
int lg_graph_build(const int64_t* edge_index, int64_t E, int64_t N,
                   int add_self_loops, int normalize, float fill_value,
                   int32_t* rowptr, int32_t* col, float* w,
                   int32_t* rowptr_t, int32_t* col_t, float* w_t,
                   void* workspace, int64_t ws_bytes, lg_stream_t stream);

/* Node table of the node-major kernels, once per graph (and once for the transposed CSR):
 * one 64-byte record per node = {e0, e1, (col, float_as_int(w)) x 6, self, node} so a tile
 * reads its CSR row with ONE scalar load.  self = position (< 6) of the row's entry whose
 * col is the node itself, -1 if none inline.  Two sections (ABI 13): records 0 .. N-1 in
 * node order, then records N .. 2N-1 in the SCHEDULE order `order` (node order[i] at
 * N + i; NULL = node order), the order in which lg_gcn_fwd_nm / lg_gcn_bwd_nm visit
 * nodes.  The order changes which tiles are in flight together, never a result: with a
 * bandwidth-reducing order (lg_rcm_order) the neighbour rows a tile gathers were gathered
 * by tiles just before it and still sit in L2.
 *   rowptr : int32 [N+1];  pairs : int32 [2 * nnz] (col, float_as_int(w));
 *   order : NULL or device int32 [N], a permutation of 0 .. N-1;
 *   nodetab : int32 [2N][16] (64-byte aligned). */
int lg_nm_table_build(const int32_t* rowptr, const int32_t* pairs, int64_t N, const int32_t* order,
                      int32_t* nodetab, lg_stream_t stream);

/* Sensor marks for the compressed layer-0 input (ABI 21; lg_node_init_bits_fwd /
 * lg_gcn_fwd_nm_x0 / lg_gcn_bwd_nm_x0).  Copies a node table (lg_nm_table_build) and its pair
 * array with every CSR entry whose col n has a sensor slot (node_slot[n] >= 0) rewritten to
 * col = 0x40000000 | node_slot[n], so a tile learns from its record alone which neighbours
 * are stored as sensor rows; pos_slot[i] = node_slot of the schedule section's record N + i.
 *   node_slot : int32 [N] (-1 = no sensor);  nodetab_out : int32 [2N][16];
 *   pairs_out : int32 [2 * nnz];  pos_slot : int32 [N]. */
int lg_nm_table_sensor_mark(const int32_t* nodetab, const int32_t* pairs, int64_t N, int64_t nnz,
                            const int32_t* node_slot, int32_t* nodetab_out, int32_t* pairs_out, int32_t* pos_slot,
                            lg_stream_t stream);

/* Reverse Cuthill-McKee order of the undirected graph edge_index (HOST memory, int64
 * [2][E], self loops and duplicates ignored): order[i] = the node visited i-th.  Each
 * connected component is a breadth-first sweep from a minimum-degree node, neighbours
 * by increasing degree (ties by id), the whole sequence reversed.  Deterministic.  Used as
 * the node-major kernels' schedule order (lg_nm_table_build): on L-TOWN-A it cuts the
 * largest |u - v| over the pipes from 656 to 27.  Returns LG_EINVAL on bad ids. */
int lg_rcm_order(const int64_t* edge_index, int64_t E, int64_t N, int32_t* order);

/* Pipe-endpoint incidence CSR, once per model (backward of detector.py:206-210).
 *   ends : int64 [P][2] device (pipe_ends, utils.py:352-358)
 *   inc_rowptr : int32 [N+1];  inc_item : int32 [2P], item = 2*p + role (role 0 = u, 1 = v),
 *   ascending item order inside each node's row. */
int64_t lg_incidence_workspace_bytes(int64_t P, int64_t N);
int lg_incidence_build(const int64_t* ends, int64_t P, int64_t N,
                       int32_t* inc_rowptr, int32_t* inc_item,
                       void* workspace, int64_t ws_bytes, lg_stream_t stream);

/* K3  disjoint-union edge index (bit-exact).
 * Replaces: detector.py:105-114 `_batchify_edge_index`:  out[:, b*E + e] = ei[:, e] + b*N.
 *   edge_index : int64 [2][E];  out : int64 [2][B*E] */
int lg_batchify_edge_index(const int64_t* edge_index, int64_t E, int64_t N, int64_t B,
                           int64_t* out, lg_stream_t stream);

/* K1+K2  node initialisation (detector.py:178-190) given the sensor projection.
 *   x0[b][n] = dropout(relu(sensor_slot[n] >= 0 ? proj[b][sensor_slot[n]] : bias))
 * where proj[b][s] = h_s[b][s] @ Ws[:, :D]^T + Ws[:, D] + bs is computed by the caller
 * (a 7,424 x 64 x 64 GEMM at B=256) and bias = bs (rows with h0 = 0, mask = 0).
 *   sensor_slot : int32 [N]  (-1 for non-sensor nodes)
 *   proj : fp32 [B][S][D];  bias : fp32 [D];  x0 : fp32 [B][N][D]
 *   flags: LG_F_DROPOUT (p, seed as lg_gcn_fwd; salt distinguishes the call site).  The
 *   keep mask is the row stream of lg_gcn_fwd_nm (seeded per window-major row b*N + n and
 *   lane group), also for lg_node_init_proj_fwd (since ABI 11; the per-element hash before). */
int lg_node_init_fwd(const int32_t* sensor_slot, const float* proj, const float* bias, float* x0,
                     int64_t B, int64_t N, int64_t S, int64_t D,
                     int flags, float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream);

/* K1+K2 with the sensor projection folded in: x0 as lg_node_init_fwd with
 *   proj[b][s] = h_s[b][s] @ W[:, :Ds]^T + W[:, Ds] + bias     (W: fp32 [D][Ds+1], nn.Linear layout)
 * formed per sensor row inside the launch (no separate GEMM / proj buffer).
 * sensor_idx: int64 [S], node of sensor s (sensor_slot is its inverse; a duplicated id's
 * earlier entries are skipped, as h0[:, idx] = h_s keeps the last write, detector.py:181).
 * Replaces: sensor_to_node (detector.py:160, 184-189) + node init.  Ds == D in {32, 64}. */
int lg_node_init_proj_fwd(const int32_t* sensor_slot, const int64_t* sensor_idx, const float* h_s, const float* W,
                          const float* bias, float* x0, int64_t B, int64_t N, int64_t S, int64_t Ds, int64_t D,
                          int flags, float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream);

/* Backward of the folded projection, from dx0 = the gradient of the node-init
 * pre-activation (lg_gcn_bwd[_nm] of layer 0 with LG_F_MASK_OUT):
 *   dproj[b][s] = dx0[row(sensor_idx[s], b)] * (live ? live[s] : 1)   (row per LG_F_NODE_MAJOR)
 *   dh_s = dproj @ W[:, :Ds];   dW = dproj^T [h_s, 1];   db = sum dproj + dbias_in (may be NULL)
 * live: fp32 [S] (0 for a duplicated sensor id whose row was overwritten, detector.py:181),
 * or NULL.  One launch + one fixed-order slab reduce (deterministic). */
int64_t lg_sensor_proj_bwd_workspace_bytes(int64_t B, int64_t S, int64_t Ds, int64_t D);
int lg_sensor_proj_bwd(const float* dx0, const int64_t* sensor_idx, const float* live, const float* h_s,
                       const float* W, const float* dbias_in, float* dh_s, float* dW, float* db, int64_t B,
                       int64_t N, int64_t S, int64_t Ds, int64_t D, int flags, void* workspace, int64_t ws_bytes,
                       lg_stream_t stream);

/* K2 backward (node init Linear(Ds+1 -> D), detector.py:160, 184-189), weight side:
 * for sensor rows the Linear input is [h_s, 1], so with dy = d(proj) [K][M] (K = B*S rows)
 * and x = h_s [K][N]:
 *   dw[m][n] = sum_k dy[k][m] x[k][n]  (n < N),   dw[m][N] = sum_k dy[k][m]
 *   db[m]    = sum_k dy[k][m]            (db may be NULL)
 * dw is [M][N+1], the nn.Linear weight layout.  M, N in {32, 64}.  Split-K over
 * workgroups, fixed-order reduction (deterministic).  Replaces the skinny-K
 * (K = 7,424) torch.mm of the autograd of torch.addmm. */
int64_t lg_linear_dw_workspace_bytes(int64_t K, int64_t M, int64_t N);
int lg_linear_dw(const float* dy, const float* x, int64_t K, int64_t M, int64_t N,
                 float* dw, float* db, void* workspace, int64_t ws_bytes, lg_stream_t stream);

/* nnz_cap (lg_gcn_fwd / lg_spmm / lg_gcn_bwd): capacity of col/w as allocated for
 * lg_graph_build (E + N).  It sizes the on-chip copy of the CSR: when
 * 4*(N+1) + 8*nnz_cap <= 48 KiB every workgroup stages the CSR in LDS once.
 *
 * K5+K6+K7  fused GCN layer forward (one launch).
 * Replaces: GCNConv.forward (lin -> propagate -> +bias, detector.py:199) and the
 * following F.relu + dropout (detector.py:200-201):
 *   y = dropout(relu( Ahat (x W^T) + b ))  computed as  (Ahat x) W^T + b
 * Each 64-lane wavefront owns 16-row tiles of a persistent, XCD-aware schedule:
 * it gathers a whole tile (CSR segmented reduce in entry order, fp32, 16 lanes per
 * row) into LDS, computes it transposed, y^T = W (Ahat x)^T, on MFMA
 * (v_mfma_f32_16x16x4_f32, exact fp32) while the next tile's row loads are in
 * flight, and applies bias/ReLU/dropout before whole-row stores.
 *   rowptr/col/w : CSR from lg_graph_build;  x, y : fp32 [B][N][D];  W : fp32 [D][D]
 *   (nn.Linear layout [out][in]);  bias : fp32 [D] or NULL.
 *   Dropout: keep element (row, c) iff hash(seed, salt, row*D + c) >= p, scale 1/(1-p).
 *   x and y must not alias. */
int lg_gcn_fwd(const int32_t* rowptr, const int32_t* col, const float* w,
               const float* x, const float* W, const float* bias, float* y,
               int64_t B, int64_t N, int64_t D, int64_t nnz_cap,
               int flags, float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream);

/* Node-major fused GCN layer (LG_F_NODE_MAJOR layout, x, y : fp32 [N][B][D]).
 * Same math, flags and results as lg_gcn_fwd on the transposed layout: rows n*B + b.
 * Every window shares the graph, so a 16-row tile is one node and 16 consecutive
 * windows, and each CSR entry (m, w) names one contiguous 16 x D block of x — the
 * entry is wave-uniform and the row loads need no per-lane index arithmetic.
 *   nodetab : int32 [2N][16] from lg_nm_table_build (one 64-byte record per node:
 *             e0, e1, the first 6 (col, w) pairs of the row, self position, node id;
 *             tiles are visited in the table's schedule order);
 *   pairs : int32 [2 * nnz] interleaved (col, float_as_int(w)) of the lg_graph_build CSR.
 *   Dropout: row-stream masks indexed by the window-major row b*N + n (the mask of
 *   lg_gcn_fwd for the same seed/salt).
 *   Requires N*B*D*4 <= 0x7FFFF000 bytes (LG_EUNSUPPORTED otherwise; callers split
 *   larger batches over windows). */
int lg_gcn_fwd_nm(const int32_t* nodetab, const int32_t* pairs, const float* x, const float* W,
                  const float* bias, float* y, int64_t B, int64_t N, int64_t D, int64_t nnz_cap,
                  int flags, float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream);
/* Backward of lg_gcn_fwd_nm: lg_gcn_bwd's contract on the node-major layout, over the
 * transposed CSR given as nodetab_t (lg_nm_table_build of rowptr_t) + pairs_t.
 * workspace: lg_gcn_bwd_nm_workspace_bytes(D). */
int64_t lg_gcn_bwd_nm_workspace_bytes(int64_t D);
int lg_gcn_bwd_nm(const int32_t* nodetab_t, const int32_t* pairs_t, const float* dy, const float* y,
                  const float* x, const float* W, float* dx_out, float* dW, float* db,
                  const int32_t* node_slot, float* dnode_bias, int64_t B, int64_t N, int64_t D,
                  int flags, float scale_in, float scale_out, void* workspace, int64_t ws_bytes, lg_stream_t stream);

/* The layer's output mask as bits (ABI 15).  lg_gcn_fwd_nm_bits = lg_gcn_fwd_nm that also
 * writes ymask (when non-NULL): [y > 0] of every output element, one uint16 per lane and
 * 16-row tile (node n, window group g = b / 16): bit 4k + i of lane l at
 * ((n * ceil(B/16) + g) * 64 + l) * 2 bytes is row g*16 + (64/(D/4)) k + l / (D/4), channel
 * 4 (l % (D/4)) + i  ->  N * ceil(B/16) * 128 bytes (1/32 of y).  lg_gcn_bwd_nm_bits =
 * lg_gcn_bwd_nm that, under LG_F_MASK_IN with ymask non-NULL, reads the mask from those
 * bits instead of gathering y (y may then be NULL).  Same results as the y path. */
/* The fp32-tier forward transform: see the LG_F_PC / LG_F_BF16X3 / LG_F_NM3 flags above. */
int lg_gcn_fwd_nm_bits(const int32_t* nodetab, const int32_t* pairs, const float* x, const float* W,
                       const float* bias, float* y, int64_t B, int64_t N, int64_t D, int64_t nnz_cap,
                       int flags, float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream,
                       uint16_t* ymask);
/* lg_gcn_bwd_nm[_bits] transform (ABI 22): on the fp32 tier both GEMMs (dx^T = W^T t^T,
 * dW = t^T x) run on the 2-way fp16 split with power-of-two scales — W^T per workgroup, each
 * 16-row tile's t and x blocks per tile — (|err| ~1e-7 of scale); LG_F_BF16X3 restores the
 * 3-way bf16 split (~1e-8).  Measured equal in time at B = 256 (the kernel is bound by its
 * gathers, not the transform); LG_F_BF16: one bf16 product. */
int lg_gcn_bwd_nm_bits(const int32_t* nodetab_t, const int32_t* pairs_t, const float* dy, const float* y,
                       const float* x, const float* W, float* dx_out, float* dW, float* db,
                       const int32_t* node_slot, float* dnode_bias, int64_t B, int64_t N, int64_t D,
                       int flags, float scale_in, float scale_out, void* workspace, int64_t ws_bytes, lg_stream_t stream,
                       const uint16_t* ymask);

/* Compressed layer-0 input (ABI 21).  The node init's non-sensor rows are dropout(relu(b)):
 * 632 of L-TOWN-A's 661 rows carry no information beyond their keep bits, yet materialising
 * x0 costs a 43 MB write and layer 0's forward and backward read it back (86 MB).
 * lg_node_init_bits_fwd replaces lg_node_init_proj_fwd (LG_F_NODE_MAJOR layout) with
 *   xs0    : fp32 [S][B][D], x0's rows of the live sensor slots (node_slot[n] = s), bit-identical
 *            to lg_node_init_proj_fwd's rows;
 *   x0bits : uint16 [N * ceil(B/16) * 64], [x0 > 0] of EVERY row in the mask layout of
 *            lg_gcn_fwd_nm_bits (ABI 15),
 * from which a non-sensor element is x0 = bit ? relu(bias) * scale : 0 exactly.
 * lg_gcn_fwd_nm_x0 is lg_gcn_fwd_nm_bits of layer 0 reading (xs0, x0bits, node_bias) through a
 * sensor-marked node table (lg_nm_table_sensor_mark): the gather waves read one 2-byte mask word
 * per neighbour block and the transform waves add the sensor neighbours' xs0 rows (ABI 22), so
 * y equals the dense forward up to that summation order (~1e-7 of scale).  lg_gcn_bwd_nm_x0 is lg_gcn_bwd_nm_bits of layer 0 (no
 * MASK_IN) with the tile's own x block from (xs0, x0bits); pos_slot_t = the transposed table's
 * schedule-section slots.  The node init and the layer share one Dropout (detector.py:190,
 * 201): flags' LG_F_DROPOUT and dropout_p describe both.  lg_node_init_expand materialises x0
 * (diagnostics, tests).  lg_gcn_fwd_nm_x0 runs on the producer / consumer kernel only: LG_F_NM3
 * and LG_F_F32_MFMA return LG_EUNSUPPORTED (ABI 25; ignored before). */
int lg_node_init_bits_fwd(const int32_t* sensor_slot, const int64_t* sensor_idx, const float* h_s, const float* W,
                          const float* bias, float* xs0, uint16_t* x0bits, int64_t B, int64_t N, int64_t S,
                          int64_t Ds, int64_t D, int flags, float dropout_p, uint64_t seed, uint32_t salt,
                          lg_stream_t stream);
int lg_node_init_expand(const int32_t* sensor_slot, const float* xs0, const uint16_t* x0bits, const float* bias,
                        float* x0, int64_t B, int64_t N, int64_t D, int flags, float dropout_p, lg_stream_t stream);
int lg_gcn_fwd_nm_x0(const int32_t* nodetab_s, const int32_t* pairs_s, const float* xs0, const uint16_t* x0bits,
                     const float* node_bias, const float* W, const float* bias, float* y, int64_t B, int64_t N,
                     int64_t S, int64_t D, int flags, float dropout_p, uint64_t seed, uint32_t salt,
                     lg_stream_t stream);
int lg_gcn_bwd_nm_x0(const int32_t* nodetab_t, const int32_t* pairs_t, const int32_t* pos_slot_t, const float* dy,
                     const float* xs0, const uint16_t* x0bits, const float* node_bias, const float* W, float* dx_out,
                     float* dW, float* db, const int32_t* node_slot, float* dnode_bias, int64_t B, int64_t N,
                     int64_t S, int64_t D, int flags, float dropout_p, float scale_out, void* workspace,
                     int64_t ws_bytes, lg_stream_t stream);

/* Single graph (B = 1) on the node tables (ABI 18): the GCNConv module's own call shape,
 * x [N][D] (BASELINE configs[4], one 100k-node graph).  Replaces: PyG GCNConv.forward
 * (detector.py:163,199 — lin, propagate, bias) and its autograd backward for ONE graph.
 * Tiles of 16 nodes in the table's schedule order; transform and dx on the 3-way bf16
 * split (fp32-level, ~1e-7 of scale), not bit-identical to lg_gcn_fwd / lg_gcn_bwd.
 *   lg_gcn_fwd_rows: y = Ahat x W^T (+ b with LG_F_BIAS; no other flags).
 *   lg_gcn_bwd_rows: t = Ahat^T dy; dx = t W; dW = t^T x; db = sum_rows dy (db may be NULL);
 *     workspace lg_gcn_bwd_nm_workspace_bytes(D).
 * D = 64 only (LG_EUNSUPPORTED otherwise: use lg_gcn_fwd / lg_gcn_bwd). */
int lg_gcn_fwd_rows(const int32_t* nodetab, const int32_t* pairs, const float* x, const float* W, const float* bias,
                    float* y, int64_t N, int64_t D, int flags, lg_stream_t stream);
int lg_gcn_bwd_rows(const int32_t* nodetab_t, const int32_t* pairs_t, const float* dy, const float* x,
                    const float* W, float* dx, float* dW, float* db, int64_t N, int64_t D, void* workspace, int64_t ws_bytes,
                    lg_stream_t stream);

/* Plain propagate y = Ahat x (PyG MessagePassing.propagate with the gcn_norm
 * weights; no transform).  Used for the HBM-roofline stress case (config C5). */
int lg_spmm(const int32_t* rowptr, const int32_t* col, const float* w,
            const float* x, float* y, int64_t B, int64_t N, int64_t D, int64_t nnz_cap, lg_stream_t stream);

/* Propagate of any width: y[n][c] = sum over row n of the CSR (entry order) of
 * w[e] x[col[e]][c], plus bias[c] when bias is non-null, for n < N, c < C (row strides ldx,
 * ldy >= C, in floats; x and y must not alias).  The general path of GCNConv (in_channels !=
 * out_channels or widths other than 32 / 64: reference detector.py:198-199 builds
 * GCNConv(hidden, hidden), PyG's GCNConv takes any pair): y = Ahat (x W^T) + b with the
 * transform on a library GEMM, or (x's width < the output's) (Ahat x) W^T + b; the backward is
 * the same call over the transposed CSR (lg_graph_build's rowptr_t / col_t / w_t).  No
 * capacity limits beyond N * C < 2^62.  (ABI 24) */
int lg_spmm_cols(const int32_t* rowptr, const int32_t* col, const float* w, const float* x, int64_t ldx,
                 const float* bias, float* y, int64_t ldy, int64_t N, int64_t C, lg_stream_t stream);

/* Fused GCN layer backward (one main launch + one deterministic slab reduction).
 * Given dy = dL/dy of this layer's output:
 *   dz     = LG_F_MASK_IN ? dy * scale_in * [y > 0] : dy
 *   t      = Ahat^T dz                     (gather over the transposed CSR)
 *   dx     = t W                           (MFMA)
 *   dW     = t^T x                         (MFMA, per-block fp32 slabs, fixed-order reduce)
 *   db     = sum_rows dz
 *   dx_out = LG_F_MASK_OUT ? dx * scale_out * [x > 0] : dx
 * Replaces: the autograd backward of GCNConv (lin, propagate, bias) and of the
 * relu/dropout pairs around it (detector.py:189-190, 198-201).
 *   dnode_bias = sum over rows b*N + n with node_slot[n] < 0 of dx_out
 *              (the node-init bias gradient, detector.py:184-190: rows without a
 *              sensor are relu(bias)); node_slot / dnode_bias both NULL to skip.
 *   y may be NULL unless LG_F_MASK_IN;  db may be NULL.
 *   workspace : lg_gcn_bwd_workspace_bytes(D) bytes. */
int64_t lg_gcn_bwd_workspace_bytes(int64_t D);
int lg_gcn_bwd(const int32_t* rowptr_t, const int32_t* col_t, const float* w_t,
               const float* dy, const float* y, const float* x, const float* W,
               float* dx_out, float* dW, float* db,
               const int32_t* node_slot, float* dnode_bias,
               int64_t B, int64_t N, int64_t D, int64_t nnz_cap,
               int flags, float scale_in, float scale_out,
               void* workspace, int64_t ws_bytes, lg_stream_t stream);

/* K8 forward: per-pipe endpoint gather + EdgeHead feature build.
 * Replaces: detector.py:206-210 and :87  feat = cat[h_u, h_v, |h_u - h_v|].
 *   ends : int64 [P][2];  h : fp32 [B][N][D];  feat : fp32 [B][P][3D] */
int lg_pipe_gather_fwd(const int64_t* ends, const float* h, float* feat,
                       int64_t B, int64_t N, int64_t P, int64_t D, lg_stream_t stream);

/* K8 backward + K10 backward, fused: deterministic segmented reduce over the
 * incidence CSR (no atomics):
 *   dh[b][n] = dpool[b]/N + sum over incidences (p, role) of n, in item order, of dpipe[b][p][role]
 * where dpipe[b][p][0] / [1] are the gradients w.r.t. h_u / h_v of pipe p (from
 * lg_edge_head_bwd).  dpool may be NULL.
 * Replaces: autograd of h_nodes[:, u], h_nodes[:, v] (detector.py:209-210) and of
 * global_mean_pool (detector.py:215).   dpipe : fp32 [B][P][2][D];  dh : fp32 [B][N][D] */
int lg_pipe_scatter_bwd(const int32_t* inc_rowptr, const int32_t* inc_item, const float* dpipe,
                        const float* dpool, float* dh,
                        int64_t B, int64_t N, int64_t P, int64_t D, int flags, lg_stream_t stream);

/* K8 + K9 fused EdgeHead forward (detector.py:76-88 applied at :206-211):
 *   logits[b][p] = W2 . dropout(relu(W1 [h_u, h_v, |h_u - h_v|] + b1)) + b2
 * feat (B,P,3D) and the hidden layer are never materialised.  W1 : fp32 [hidden][3D]
 * (edge_head.mlp.0.weight), b1 [hidden], W2 [hidden] (mlp.3.weight), b2 [1];
 * logits : fp32, element (b, p) at logits[b*ldo + p] (ldo >= P; ldo = P+1 writes the
 * pipe columns of detector.py:216's (B, P+1) output in place).  hidden must be 128;
 * D in {32, 64}.  Dropout as lg_gcn_fwd, index (b*P + p)*hidden + unit.
 * hid: NULL, or fp32 [B*P][hidden] receiving the post-dropout hidden layer (what
 * lg_edge_head_bwd needs; pass it in training).  The products run on f16 MFMA with
 * 2-way split, power-of-two-scaled fp32 operands (D = 64, fp32 tier; W1 scaled per wave,
 * the features per pipe row, dropped term <= 2^-22 of each product) or, with
 * LG_F_BF16X3 and at D = 32, on bf16 MFMA with 3-way split operands: fp32-level
 * accuracy either way, not bit-identical to an fp32 GEMM.  LG_F_BF16: bf16 hi parts only. */
int lg_edge_head_fwd(const int64_t* ends, const float* h, const float* w1, const float* b1,
                     const float* w2, const float* b2, float* logits, int64_t ldo, float* hid,
                     int64_t B, int64_t N, int64_t P, int64_t D, int64_t hidden,
                     int flags, float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream);
/* Backward of lg_edge_head_fwd: hid (its hidden-layer output) and dlogits (row stride
 * ldo) -> dpipe fp32 [B][P][2][D] (grads w.r.t. h_u, h_v per pipe), dw1/db1/dw2/db2
 * (overwritten; deterministic fixed-order reduction of per-workgroup slabs).  flags and
 * dropout_p as in the forward (the keep mask is read back as [hid > 0]).  Transform (ABI
 * 22): on the fp32 tier the f16x2 split — g rows scaled per pipe row from |dlogit| (dpipe
 * independent of which rows share a tile), W1^T per wave, dW1's products per tile (features
 * scaled by 2^(T - sg(row))); LG_F_BF16X3: the 3-way bf16 split; LG_F_BF16: one product. */
int64_t lg_edge_head_bwd_workspace_bytes(int64_t B, int64_t P, int64_t D, int64_t hidden);
int lg_edge_head_bwd(const int64_t* ends, const float* h, const float* w1, const float* w2,
                     const float* hid, const float* dlogits, int64_t ldo, float* dpipe,
                     float* dw1, float* db1, float* dw2, float* db2,
                     int64_t B, int64_t N, int64_t P, int64_t D, int64_t hidden,
                     int flags, float dropout_p, void* workspace, int64_t ws_bytes, lg_stream_t stream);
/* lg_edge_head_bwd followed by lg_pipe_scatter_bwd (dh = dpool / N + the incidence sums of
 * dpipe; reference detector.py:206-211 and the backward of its gather), fused into the
 * backward kernel.  With a pipe schedule (sched: device copy of lg_pipe_schedule_build's
 * buffer, sched_hdr: its first 16 words in HOST memory; ABI 22) the node sums are STREAMED:
 * pipes are visited in the schedule's order, each tile's per-pipe rows stay in LDS and are
 * added to the running sums of the nodes they touch (LDS slots for the nodes still open, the
 * dh row at a node's last tile) — dpipe is neither written nor read.  The sums are those of
 * lg_pipe_scatter_bwd over the schedule's incidence CSR (inc_rowptr / inc_item from the same
 * build), bit for bit.  Without a schedule (NULL, NULL), or when the open sums do not fit in
 * LDS, each workgroup owns whole windows and sums a window's node rows from its just-written
 * dpipe rows (ABI 19; the CSR staged in LDS), or, when the CSR does not fit either, the two
 * calls run.  Both fused forms run one workgroup per window, so with fewer windows (B) than
 * CUs the two calls run instead.  dpipe: scratch [B][P][2][D] (untouched by the streamed path); dpool: NULL or
 * [B][D] (lg_pool_head_bwd's dpooled, computed before this call); the workspace is
 * lg_edge_head_bwd_workspace_bytes.  A schedule for another (P, N, D) is LG_EINVAL. */
int lg_edge_head_bwd_scatter(const int64_t* ends, const float* h, const float* w1, const float* w2,
                             const float* hid, const float* dlogits, int64_t ldo, float* dpipe,
                             float* dw1, float* db1, float* dw2, float* db2, const int32_t* inc_rowptr,
                             const int32_t* inc_item, const int32_t* sched, const int32_t* sched_hdr,
                             const float* dpool, float* dh,
                             int64_t B, int64_t N, int64_t P, int64_t D, int64_t hidden,
                             int flags, float dropout_p, void* workspace, int64_t ws_bytes, lg_stream_t stream);

/* Both heads' backward (ABI 23): lg_pool_head_bwd (the NoLeakHead, first argument block) then
 * lg_edge_head_bwd_scatter, as ONE launch when the streamed form applies (a pipe schedule, a
 * window per workgroup): the NoLeakHead backward of each workgroup's windows runs in its
 * prologue (the same sums in the same order as k_pool_head_bwd), dpool [B][D] becomes a scratch
 * the launch writes and reads back.  Otherwise the two calls, in that order (dpool their
 * hand-off).  nworkspace: lg_pool_head_bwd_workspace_bytes; workspace:
 * lg_edge_head_bwd_workspace_bytes.  Replaces detector.py:214-216's and :206-211's autograd
 * (global_mean_pool + NoLeakHead, pipe gather + EdgeHead). */
int lg_heads_bwd_scatter(const float* pooled, const float* nhid, const float* nw1, const float* nw2, float* ndw1,
                         float* ndb1, float* ndw2, float* ndb2, int nflags, float n_dropout_p, void* nworkspace,
                         int64_t nws_bytes, const int64_t* ends, const float* h, const float* w1, const float* w2,
                         const float* hid, const float* dlogits, int64_t ldo, float* dpipe, float* dw1, float* db1,
                         float* dw2, float* db2, const int32_t* inc_rowptr, const int32_t* inc_item,
                         const int32_t* sched, const int32_t* sched_hdr, float* dpool, float* dh, int64_t B, int64_t N,
                         int64_t P, int64_t D, int64_t hidden, int flags, float dropout_p, void* workspace,
                         int64_t ws_bytes, lg_stream_t stream);

/* Pipe schedule of the streamed EdgeHead backward (ABI 22), once per model; HOST memory in and
 * out (upload sched to the device; keep its first 16 words on the host as sched_hdr).
 *   ends : int64 [P][2];  D : 32 or 64 (the tile height 2048 / D);
 *   sched : int32 [words] with words >= lg_pipe_schedule_words(P, N, D);
 *   inc_rowptr [N+1], inc_item [2P]: the incidence CSR (as lg_incidence_build) with each node's
 *     items in SCHEDULE order instead of ascending — pass it to lg_pipe_scatter_bwd /
 *     lg_edge_head_bwd_scatter with this schedule, so every path sums in one order.
 * Pipes are ordered by their endpoints' positions in lg_rcm_order of the pipe graph (the later
 * one first, then the earlier, then the id); a node is "open" from its first tile to its last.
 * Header words: version, P, N, D, TR, tiles, open slots, max events per tile, block words,
 * nodes without pipes, the three section offsets, total words.  Deterministic.
 * LG_EUNSUPPORTED when N >= 2^24. */
#define LG_PIPE_SCHED_VERSION 1
int64_t lg_pipe_schedule_words(int64_t P, int64_t N, int64_t D);
int lg_pipe_schedule_build(const int64_t* ends, int64_t P, int64_t N, int64_t D, int32_t* sched, int64_t words,
                           int32_t* inc_rowptr, int32_t* inc_item);

/* K10 forward: per-window mean over the N node rows.
 * Replaces: global_mean_pool(x, batch) with batch = arange(B).repeat_interleave(N)
 * (detector.py:214-215).   x : fp32 [B][N][D];  out : fp32 [B][D] */
int lg_mean_pool_fwd(const float* x, float* out, int64_t B, int64_t N, int64_t D, lg_stream_t stream);

/* K10 + NoLeakHead fused (detector.py:91-102 applied at :214-216):
 *   pooled[b] = mean_n x[b][n]                                  (global_mean_pool)
 *   hid[b]    = dropout(relu(pooled[b] W1^T + b1))              (noleak_head.mlp.0-2)
 *   logits[b*ldo + col] = hid[b] . w2 + b2                      (mlp.3, squeeze)
 * x : fp32 [B][N][D];  w1 [hidden][D], b1 [hidden], w2 [hidden], b2 [1];
 * pooled [B][D] and hid [B][hidden] are outputs saved for the backward.  hidden must
 * be 128; D in {32, 64}; dropout index b*hidden + unit.  With col = P and ldo = P+1
 * this writes the no-leak column of the (B, P+1) logits in place. */
int lg_pool_head_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                     float* pooled, float* hid, float* logits, int64_t ldo, int64_t col,
                     int64_t B, int64_t N, int64_t D, int64_t hidden,
                     int flags, float dropout_p, uint64_t seed, uint32_t salt, lg_stream_t stream);
/* Backward: dlogits[b*ldo + col] -> dpooled fp32 [B][D] (pass to lg_pipe_scatter_bwd as
 * dpool), dw1/db1/dw2/db2 (overwritten; deterministic; db2 summed in fp64).  The ReLU /
 * dropout masks are read back from hid (> 0), scaled by 1/(1-p) under LG_F_DROPOUT. */
int64_t lg_pool_head_bwd_workspace_bytes(int64_t B, int64_t D, int64_t hidden);
int lg_pool_head_bwd(const float* pooled, const float* hid, const float* w1, const float* w2,
                     const float* dlogits, int64_t ldo, int64_t col, float* dpooled,
                     float* dw1, float* db1, float* dw2, float* db2,
                     int64_t B, int64_t D, int64_t hidden, int flags, float dropout_p,
                     void* workspace, int64_t ws_bytes, lg_stream_t stream);

/* ---------------------------------------------------------------------------
 * SharedSensorGRUEncoder (detector.py:28-73): one nn.GRU(1 [+9], H) over the
 * B*S sensor sequences (q = b*S + s), L steps, output h_L.  PyTorch gate order
 * (r, z, n) and formulas; weights in nn.GRU layout (weight_ih_l0 [3H][I],
 * weight_hh_l0 [3H][H]).  x_t = [residual[b][t][s], tfeat[b][t][0..8]] is read in
 * place — the (B*S, L, 10) concatenation of detector.py:62-67 is never built.
 *   residual : fp32 [B][L][S];  tfeat : fp32 [B][L][9] (I = 10) or NULL (I = 1)
 *   h_seq    : fp32 [L][B*S][H] every step's h (for the backward) or NULL
 *   gates    : fp32 [L][B*S][4][H] per step (r, z, n, W_hn h + b_hn) for the
 *              backward, or NULL (inference); non-NULL requires h_seq
 *   h_last   : fp32 [B*S][H]  (= h_s of detector.py:176 as [B][S][H])
 * H in {32, 64} on the tiled kernels below; any other H in 1..1024 (ABI 26; LG_EUNSUPPORTED
 * before) on a generic kernel (one hidden unit per thread, fp32 FMAs, same saved layouts: a
 * generality path for LeakDetector(sensor_hidden=...), not the bench's).  I in {1, 10}
 * (use_time False/True), one layer.
 * Backward (BPTT from the saved gates, no recompute): dh_last -> dx (fp32
 * [B*S][L][I], may be NULL), dW_ih, dW_hh, db_ih, db_hh (overwritten,
 * deterministic).
 * Precision (round 4): the recurrent products of the forward and of the dx == NULL backward
 * run on the f16x2 split (two f16 parts, power-of-two scales, fp32 accumulate: |error| <=
 * 2^-22 of each product); the backward's dG scale follows a bound on the previous step's
 * maxima, so gradients of any magnitude keep that accuracy (tests/test_gpu_parity.py
 * test_gru_bwd_f16x2_scales).  The dx != NULL backward stays on fp32 MFMA. */
int lg_gru_fwd(const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
               const float* b_ih, const float* b_hh, float* h_seq, float* gates, float* h_last,
               int64_t B, int64_t L, int64_t S, int64_t I, int64_t H, lg_stream_t stream);
int64_t lg_gru_bwd_workspace_bytes(int64_t B, int64_t S, int64_t I, int64_t H);
int lg_gru_bwd(const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
               const float* h_seq, const float* gates, const float* dh_last,
               float* dx, float* dw_ih, float* dw_hh, float* db_ih, float* db_hh,
               int64_t B, int64_t L, int64_t S, int64_t I, int64_t H,
               void* workspace, int64_t ws_bytes, lg_stream_t stream);

/* The GRU encoder and the node init in one launch each way (ABI 23; the node-major trunk's
 * compressed node init, lg_node_init_bits_fwd, with the sensor projection's backward,
 * lg_sensor_proj_bwd).  Replaces detector.py:60-73 (the shared GRU) followed by :179-190 (h0,
 * the mask column, sensor_to_node, ReLU, dropout) when node_hidden == sensor_hidden == H.
 *   fwd: lg_gru_fwd's outputs, plus xs0 [S][B][H] and x0bits exactly as lg_node_init_bits_fwd
 *        writes them from h_last (W = proj_w [H][H + 1], bias = node_bias, dropout stream =
 *        (seed, salt)), except that the sensor nodes' words of x0bits are 0 (no reader:
 *        lg_gcn_fwd_nm_x0 / lg_gcn_bwd_nm_x0 take those rows from xs0).  One launch.
 *   bwd: lg_gru_bwd without dx, its dh_last formed in the launch from the node init's
 *        pre-activation gradient, as lg_sensor_proj_bwd does: dx0 is node-major [N][B][H] (the
 *        sensor nodes' rows: lg_gcn_bwd_nm_x0 with LG_F_DX_SENSOR_ROWS), live [S] (may be NULL);
 *        also dproj_w [H][H + 1] and dproj_b [H] (+ dbias_in, the non-sensor rows' sum, which
 *        may be a pending output of an open reduce batch).  One launch + one slab reduction of
 *        all six gradients.  Workspace: lg_gru_node_init_bwd_workspace_bytes. */
int lg_gru_node_init_fwd(const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
                         const float* b_ih, const float* b_hh, float* h_seq, float* gates, float* h_last,
                         const int32_t* sensor_slot, const int64_t* sensor_idx, const float* proj_w,
                         const float* node_bias, float* xs0, uint16_t* x0bits, int64_t B, int64_t L, int64_t S,
                         int64_t I, int64_t H, int64_t N, int flags, float dropout_p, uint64_t seed, uint32_t salt,
                         lg_stream_t stream);
int64_t lg_gru_node_init_bwd_workspace_bytes(int64_t B, int64_t S, int64_t I, int64_t H);
int lg_gru_node_init_bwd(const float* residual, const float* tfeat, const float* w_ih, const float* w_hh,
                         const float* h_seq, const float* gates, const float* dx0, const int64_t* sensor_idx,
                         const float* live, const float* proj_w, const float* dbias_in, float* dw_ih, float* dw_hh,
                         float* db_ih, float* db_hh, float* dproj_w, float* dproj_b, int64_t B, int64_t L, int64_t S,
                         int64_t I, int64_t H, int64_t N, void* workspace, int64_t ws_bytes, lg_stream_t stream);

/* ---- Frozen-predictor residual builder (SURVEY 8 f rank 1) ----------------------
 * Replaces the per-window NormalPredictorTCN passes of
 * build_residual_sequence_from_segment (reference models/utils.py:169-216, TCN
 * models/predictor.py:17-81) with ONE pass per segment over the shared-window row plan
 * of models/tcn_plan.py: output row r of a conv layer reads input rows plan[r].x/.y/.z
 * (taps t, t-d, t-2d; -1 = zero padding) and, for a block's second conv, adds block-input
 * row plan[r].w (-1 = none).  Rows are segment-local; tensors are [nseg][rows][C].
 * C must be 128 (the TCN default, LG_EUNSUPPORTED otherwise); rows_out <= 2048.
 *   lg_tcn_pack_weight   Conv1d weight [C][C][3] -> packed fragment order
 *                        (lg_tcn_packed_weight_floats(C) floats), once per weight.
 *   lg_tcn_conv_fwd      y = LayerNorm(conv(x) + bias) -> ReLU (-> + residual), exact
 *                        fp32 (MFMA f32); blk = NULL for a block's first conv.  */
int64_t lg_tcn_packed_weight_floats(int64_t C);
int lg_tcn_pack_weight(const float* weight, float* packed, int64_t C, lg_stream_t stream);
int lg_tcn_conv_fwd(const float* in, const float* blk, const int32_t* plan, const float* packed_weight,
                    const float* bias, const float* ln_w, const float* ln_b, float eps, float* out,
                    int64_t nseg, int64_t rows_in, int64_t rows_blk, int64_t rows_out, int64_t C,
                    lg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* LEAKGNN_H */
