/*
 * hmmbw.h — C ABI of the MI355X-native Baum-Welch engine (libhmmbw.so).
 *
 * The reference (DemianMArin/HMM_Training, pure Python/NumPy) has no FFI; its hot-path boundary is
 * the Python function
 *     hmm_training(observations, N=4, M=256, epsilon=1e-6, max_iterations=100,
 *                  show_progress=True, word_name=None, load_initial_params=True) -> (A, B, pi)
 * at HMM/hmm_training.py:265-267, its forward-only scorer
 *     calculate_log_likelihood(recording_observations, hmm) -> float   (HMM/hmm_testing.py:49)
 * and its VQ encoder get_observations (HMM/hmm_training.py:82-120).  Each entry point below says
 * which part of those functions it replaces.  The Python drop-in (hmm_training_amd/) binds this
 * ABI with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Every function returns an int status: HMMBW_OK (0) or a negative HMMBW_E_* code; the message
 *    of the last failure on the calling thread is hmmbw_last_error().  No C++ exception crosses
 *    the ABI.
 *  - All arrays are plain row-major host or device pointers with explicit sizes; no torch types.
 *  - Probabilities are fp64, LINEAR domain (the reference converts with safe_log/safe_exp at
 *    hmm_training.py:323-325 and :524-526; the engine's scaled-linear recursions are the same
 *    quantities).
 *  - Work is enqueued on the context's HIP stream (hmmbw_set_stream) and is asynchronous, except
 *    the functions marked SYNC, which synchronise that stream.
 *  - One context per device per thread; contexts are independent.
 */
#ifndef HMMBW_H
#define HMMBW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HMMBW_ABI_VERSION 5 /* 2: hmmbw_iterate_begin/_end, status snapshots, comm info/payload;
                              3: peer all-reduce (hmmbw_peer_*), HMMBW_E_TIMEOUT, cache trim, split timing;
                              4: live status mirror (HMMBW_OPT_LIVE_STATUS, hmmbw_status_live_wait);
                              5: hmmbw_get_option, HMMBW_OPT_WQ_TIMEOUT_MS, HMMBW_OPT_WIDE_WQ */

#define HMMBW_OK 0
#define HMMBW_E_INVALID (-1)        /* bad argument (shape, range, null pointer)             */
#define HMMBW_E_HIP (-2)            /* HIP runtime error                                      */
#define HMMBW_E_UNSUPPORTED (-3)    /* shape outside what the kernels implement (N > 64)       */
#define HMMBW_E_STATE (-4)          /* call order violated (e.g. estep before observations)   */
#define HMMBW_E_EMPTY_SEQUENCE (-5) /* a sequence of length 0: the reference raises IndexError
                                       at hmm_training.py:376 / hmm_testing.py:75              */
#define HMMBW_E_SYMBOL_RANGE (-6)   /* symbol id >= M: numpy IndexError at hmm_training.py:360 */
#define HMMBW_E_TIMEOUT (-7)        /* a bounded device-side wait expired: a rank did not deliver its
                                       statistics to the peer all-reduce in time, or a wide work-queue
                                       backward sweep did not see its forward finish (EM stops, the
                                       status calls report it; hmmbw_last_error says which)           */

/* Transition-matrix kernel variant (the reference skips -inf transitions,
 * hmm_training.py:143-144,186-188; a left-to-right A keeps its zero pattern under EM). */
#define HMMBW_TOPOLOGY_AUTO 0          /* left-to-right if A's zero pattern allows, else dense */
#define HMMBW_TOPOLOGY_DENSE 1
#define HMMBW_TOPOLOGY_LEFT_TO_RIGHT 2 /* a_ij == 0 unless j in {i, i+1}                      */

typedef struct hmmbw_ctx hmmbw_ctx;

/* One EM iteration's convergence record: hmm_training.py:503-513 (L = LSE_r log P_r of the
 * parameters ENTERING the iteration, diff = |L - L_prev| or +inf on the first iteration). */
typedef struct {
    double log_likelihood;
    double diff;
} hmmbw_iter_record;

typedef struct {
    int64_t iterations; /* EM iterations executed (the reference's `iteration`, :514)          */
    int32_t done;       /* 1 once `diff >= epsilon and iteration < max_iterations` (:346) fails */
    int32_t converged;  /* 1 if it stopped on epsilon rather than on max_iterations (:516-521)  */
    double last_log_likelihood;
    double last_diff;
} hmmbw_status;

int hmmbw_abi_version(void);
const char *hmmbw_last_error(void);
int hmmbw_device_count(int *out);

/* The library keeps the small device buffers and pinned snapshot blocks of destroyed contexts (blocks
 * <= 4 MB, at most 32 MB per kind and device) for the next context: the drop-in builds one context per
 * hmm_training call (hmm_training.py:265-267) and hipFree synchronises the device.  This returns every
 * cached block to the driver (e.g. before a memory-hungry phase of the process, or on an
 * out-of-memory); *bytes_released (may be NULL) gets the total.  Blocks of live contexts are not
 * touched. */
int hmmbw_cache_trim(int64_t *bytes_released);

/* Context for one (device, N states, M symbols) model.  Replaces the parameter set-up of
 * hmm_training.py:268-339 (allocation is sized by hmmbw_set_observations). */
int hmmbw_ctx_create(int device, int n_states, int n_symbols, hmmbw_ctx **out);
int hmmbw_ctx_destroy(hmmbw_ctx *ctx);
int hmmbw_set_stream(hmmbw_ctx *ctx, void *hip_stream); /* hipStream_t; NULL = legacy default */
int hmmbw_set_rank(hmmbw_ctx *ctx, int rank, int world_size);
int hmmbw_set_topology(hmmbw_ctx *ctx, int topology);
int hmmbw_get_topology(const hmmbw_ctx *ctx, int *out); /* resolved variant (after AUTO)      */

/* Observation sequences as host CSR: sequence r is symbols[offsets[r] .. offsets[r+1]).
 * Replaces the `observations: List[np.ndarray]` argument (hmm_training.py:265) — the caller
 * keeps ownership; the library copies to HBM in its own length-sorted, time-major layout. */
int hmmbw_set_observations(hmmbw_ctx *ctx, const int64_t *offsets, const int32_t *symbols, int64_t n_seq);

/* Linear (pi[N], A[N*N], B[N*M]) host arrays: the initial parameters (hmm_training.py:299-325). */
int hmmbw_set_params(hmmbw_ctx *ctx, const double *pi, const double *A, const double *B);

/* Arm a training run: epsilon and max_iterations of hmm_training.py:265-266,342-346. */
int hmmbw_reset_training(hmmbw_ctx *ctx, double epsilon, int64_t max_iterations);

/* Length (in doubles) of the packed sufficient-statistics buffer used by estep/mstep. */
int hmmbw_stats_len(const hmmbw_ctx *ctx, int64_t *n_doubles);

/* E-step over this rank's sequences (hmm_training.py:351-410): writes this rank's packed statistics
 * {pi_num[N], xi[N*N], gamma_den_excl_last[N], gamma_den_all[N], B_num[M*N], (m, s)[world]}
 * (linear-domain sums: xi_ij = sum_r sum_t xi_t(i,j), B_num symbol-major [M][N]) into the DEVICE
 * buffer stats_dev (hmmbw_stats_len doubles; its (m, s) pair — the max and sum-exp of log P_r —
 * in slot `rank`, other slots zero).  Multi-rank callers all-reduce(sum) stats_dev, then call
 * hmmbw_mstep.  A deferred M-step (below) runs at the start of this launch. */
int hmmbw_estep(hmmbw_ctx *ctx, double *stats_dev);

/* M-step + convergence (hmm_training.py:415-514) from the (all-reduced) statistics; n_seq_global
 * is the R of :424.  No-op once done.  With HMMBW_OPT_MERGE_MSTEP (default) it is DEFERRED: the
 * next hmmbw_estep runs it in the prologue of its own kernel, so stats_dev must stay untouched until
 * then; hmmbw_get_status / get_params / score / set_params / reset_training complete it first. */
int hmmbw_mstep(hmmbw_ctx *ctx, double *stats_dev, int64_t n_seq_global);

/* Enqueue n_iter iterations of (estep, mstep) with internal statistics (the last M-step stays
 * deferred until a query, as for hmmbw_mstep).  Iterations after convergence are device-side no-ops
 * (same result as stopping, :346).  Single rank, or several ranks with hmmbw_comm_init (below). */
int hmmbw_iterate(hmmbw_ctx *ctx, int64_t n_iter);

/* Native RCCL communicator for the multi-rank loop.  With it, hmmbw_iterate(ctx, n) on a context of
 * world_size > 1 runs n iterations of {estep -> ncclAllReduce(sum) of the packed statistics on the
 * context's stream -> mstep} with no host round trip, replacing the per-iteration
 * torch.distributed.all_reduce hop (one RCCL all-reduce per EM iteration either way).  rccl_path:
 * the RCCL library the process already uses (torch's librccl.so), or NULL to look it up.  Rank 0
 * calls hmmbw_comm_unique_id and shares the 128-byte id (e.g. torch.distributed.broadcast); then
 * every rank calls hmmbw_comm_init (collective: all ranks must call it) after hmmbw_set_rank.
 * n_seq_global is the R of hmm_training.py:424 over all ranks.  (A 1-rank communicator is allowed:
 * hmmbw_iterate then takes the same multi-rank sequence, which is how it is tested on one GPU.) */
int hmmbw_comm_probe(const char *rccl_path); /* HMMBW_OK if the RCCL entry points resolve (local check) */
int hmmbw_comm_unique_id(const char *rccl_path, void *id_out);
int hmmbw_comm_init(hmmbw_ctx *ctx, const char *rccl_path, const void *id, int rank, int world_size,
                    int64_t n_seq_global);
/* SYNC. The engine communicator as created: *n_ranks = ncclCommCount (0 without a communicator),
 * plus the HIP-event time of the ncclAllReduce calls hmmbw_iterate enqueued while E-step timing was
 * on (hmmbw_timing; the same every-k-th schedule), summed in *total_ms over *count calls.  reset=1
 * clears the accumulated time.  Measurement only (bench.py's all-reduce microseconds per iteration). */
int hmmbw_comm_info(hmmbw_ctx *ctx, int *n_ranks, double *total_ms, int64_t *count, int reset);

/* Length in doubles of the last all-reduce hmmbw_iterate enqueued on the engine communicator (0
 * before the first): the fused small path all-reduces its statistics copies plus one (max, sum exp)
 * pair per rank, 256-B aligned; the other paths the packed statistics (hmmbw_stats_len). */
int hmmbw_comm_payload(const hmmbw_ctx *ctx, int64_t *n_doubles);

/* One multi-rank EM iteration split at its all-reduce, for callers that bring their own collective
 * (torch.distributed, MPI, an in-process sum over several contexts) or test the exact enqueue
 * sequence an RCCL run makes without RCCL: hmmbw_iterate_begin enqueues this rank's E-step (on the
 * small kernels the fused one that accumulates straight into the all-reduce buffer and writes the
 * rank's (max, sum exp) pair of log P; elsewhere hmmbw_estep into the packed statistics) and returns
 * the DEVICE buffer *buf of *n_doubles doubles that the caller must all-reduce (sum, in place, ordered
 * after the context's stream) before hmmbw_iterate_end, which enqueues the M-step + convergence step
 * (hmm_training.py:415-514; merged into the next E-step launch when it can).  n_seq_global is the R of
 * :424.  The buffer layout does not depend on the shard, so every rank (an empty shard too) passes the
 * same length.  hmmbw_iterate on a context with hmmbw_comm_init runs exactly begin -> ncclAllReduce ->
 * end per iteration.  Any other training call between the two returns HMMBW_E_STATE. */
int hmmbw_iterate_begin(hmmbw_ctx *ctx, int64_t n_seq_global, double **buf, int64_t *n_doubles);
int hmmbw_iterate_end(hmmbw_ctx *ctx);

/* ---- Peer all-reduce (HMMBW_OPT_ALLREDUCE = HMMBW_ALLREDUCE_PEER) ----
 * The sums the reference forms over all recordings (pi over the global R, hmm_training.py:415-424; A and B,
 * :429-500; L over all sequences, :503) are one elementwise sum of every rank's statistics buffer per EM
 * iteration.  Instead of an RCCL all-reduce, every rank owns a RECEIVE REGION in its HBM with one slot per
 * rank (double-buffered by iteration parity) and one flag per (rank, 2 KB chunk): after its E-step a rank
 * writes its buffer into slot `rank` of every rank's region (system-scope write-through stores over xGMI,
 * then the chunk's flag = the iteration's sequence number), and before its M-step it waits for all the
 * flags of its own region (bounded: HMMBW_OPT_PEER_TIMEOUT_MS) and sums the slots in rank order, so every
 * rank holds bitwise-identical sums and takes the same stop decision (:346).  Set-up, collective over the
 * ranks (all call it, after hmmbw_set_rank and the options, before the first iteration):
 *   hmmbw_peer_region     allocate this rank's receive region (*bytes; *region its device address);
 *   hmmbw_peer_ipc_handle its 64-byte HIP IPC handle, to be exchanged between the rank processes;
 *   hmmbw_peer_open       map every other rank's region from the exchanged handles (world x 64 bytes, in
 *                         rank order) and attach them, or
 *   hmmbw_peer_attach     attach regions already addressable here (world device pointers, rank order;
 *                         several ranks in one process on one GPU, as the tests run it).
 * n_seq_global is the R of hmm_training.py:424 over all ranks (hmmbw_iterate's loop).  Attaching clears
 * the flags: every rank must attach before any rank starts an iteration. */
int hmmbw_peer_region(hmmbw_ctx *ctx, void **region, int64_t *bytes);
int hmmbw_peer_ipc_handle(hmmbw_ctx *ctx, void *handle_out);
int hmmbw_peer_open(hmmbw_ctx *ctx, const void *handles, int64_t n_seq_global);
int hmmbw_peer_attach(hmmbw_ctx *ctx, void *const *regions, int64_t n_seq_global);
/* The all-reduce hmmbw_iterate and hmmbw_iterate_begin/_end use now: -1 none (single rank), 0 RCCL
 * (engine communicator, or the caller's collective for _begin/_end), 1 peer. */
int hmmbw_allreduce_kind(const hmmbw_ctx *ctx, int *kind);

/* SYNC. Status plus the iteration records [first, first+count) (ring of 4096 entries). */
int hmmbw_get_status(hmmbw_ctx *ctx, hmmbw_status *status, hmmbw_iter_record *records, int64_t first,
                     int64_t count);

/* ASYNC. Snapshot the status and the iteration records [first, iterations) on the context stream
 * into pinned host memory (one small kernel; no M-step flush: with merged M-steps the snapshot covers
 * every iteration enqueued before it except the last) and return its ticket.  Lets a host loop keep the next chunk of iterations
 * queued while it reads the previous chunk's status (the drop-in train loop, hmm_training.py
 * :346-514; iterations enqueued past convergence are device-side no-ops).  Two snapshots are kept:
 * posting a third first waits for the oldest to land. */
int hmmbw_status_post(hmmbw_ctx *ctx, int64_t first, int64_t *ticket);

/* Waits for snapshot `ticket` (one of the last two posted) only, not for the work queued after it;
 * then fills status and the records [first, first+count), which must lie inside the snapshot's
 * [first posted, iterations). */
int hmmbw_status_wait(hmmbw_ctx *ctx, int64_t ticket, hmmbw_status *status, hmmbw_iter_record *records,
                      int64_t first, int64_t count);

/* With HMMBW_OPT_LIVE_STATUS = 1 every M-step that records an iteration (:503-514) also writes that
 * record and the new status into pinned host memory from the device, while the launch that runs it (with
 * merged M-steps: the next E-step, in its prologue) is still executing.  This waits, by polling that
 * memory, until `iterations` iterations are recorded or EM has stopped, then fills status and the records
 * [first, first+count).  No stream synchronisation and no extra kernel: a host loop sees iteration e's
 * convergence record a few microseconds into launch e + 1, while launch e + 2 can already be queued
 * behind it (the reference's per-iteration check, :346,503-514, without idling the GPU).  If the stream
 * runs dry first (the last M-step still pending, or a device-side stop), it returns the device status. */
int hmmbw_status_live_wait(hmmbw_ctx *ctx, int64_t iterations, hmmbw_status *status, hmmbw_iter_record *records,
                           int64_t first, int64_t count);

/* SYNC. Current parameters.  normalise=1 applies the reference's return path (safe_exp then
 * pi/sum(pi), row-normalise A and B rows with positive sums, :524-541); normalise=0 returns the
 * unnormalised working parameters (exp of the reference's log_pi/log_a/log_b matrices). */
int hmmbw_get_params(hmmbw_ctx *ctx, double *pi, double *A, double *B, int normalise);

/* SYNC. log P(O_r | lambda) of the last E-step, in the caller's sequence order (:375-377). */
int hmmbw_get_loglik(hmmbw_ctx *ctx, double *out);

/* SYNC. Forward-only scoring of the loaded sequences under the current parameters:
 * hmm_testing.py:49-104 calculate_log_likelihood for every sequence, one launch. */
int hmmbw_score(hmmbw_ctx *ctx, double *out);

/* Engine knobs.  HMMBW_OPT_SAFE_SCALING = 1 forces the per-step power-of-two normalisation of the
 * forward recursion (default 0: lagged normalisation, automatic per-wave fallback to the per-step
 * form when magnitudes leave [2^-900, 2^900]).  Results agree to fp64 rounding either way. */
#define HMMBW_OPT_SAFE_SCALING 1
/* Diagnostics only (profiling ablations; results are WRONG while nonzero): bit 0 skips the E-step's
 * statistics flush, bit 1 skips its backward sweep, bit 2 skips the separate (unmerged) M-step kernel. */
#define HMMBW_OPT_ABLATE 2
/* Number of statistics accumulator copies the E-step's workgroups spread their atomics over
 * (workgroup b adds into copy b % n; default 2). */
#define HMMBW_OPT_STAT_COPIES 3
/* 1 (default): every M-step runs in the prologue of the next E-step launch, computed redundantly by
 * each workgroup straight into its LDS tables (when the emission tables fit LDS); 0: a separate
 * one-workgroup M-step kernel after every E-step. */
#define HMMBW_OPT_MERGE_MSTEP 4
/* 1: deterministic-reduction mode, bitwise-identical results run to run (no floating-point atomics):
 * gamma goes to per-position rows summed per symbol in a fixed order, and the other statistics are
 * per-workgroup partials summed in workgroup order.  About twice the E-step time on the small
 * kernels; the wide path (16 < N <= 64) already gathers gamma rows, so there it only replaces the
 * other statistics' atomics.  Small state counts need the LDS emission tables (HMMBW_E_UNSUPPORTED
 * otherwise); set it before hmmbw_set_observations (HMMBW_E_STATE after).  Default 0. */
#define HMMBW_OPT_DETERMINISTIC 7
/* Multi-rank all-reduce of the per-iteration statistics: 0 (default) = RCCL (hmmbw_comm_init) or the
 * caller's collective between hmmbw_iterate_begin and _end; 1 = the engine's own peer all-reduce
 * (hmmbw_peer_* below; then _begin/_end do the whole exchange and the caller adds nothing between). */
#define HMMBW_OPT_ALLREDUCE 8
#define HMMBW_ALLREDUCE_RCCL 0
#define HMMBW_ALLREDUCE_PEER 1
/* Bound, in milliseconds, of the peer all-reduce's device-side wait for the other ranks' statistics
 * (default 30000).  Past it the iteration fails with HMMBW_E_TIMEOUT instead of spinning. */
#define HMMBW_OPT_PEER_TIMEOUT_MS 9
/* 1: keep a host mirror of the convergence state that the M-steps update (hmmbw_status_live_wait);
 * 0 (default): off.  Synchronises the context stream when changed. */
#define HMMBW_OPT_LIVE_STATUS 10
/* Bound, in milliseconds, of the wide work queue's device-side wait (16 < N <= 64 with many tiles per CU,
 * HMMBW_OPT_WIDE_WQ): a backward sweep waits for its tile's forward sweep, which runs on a resident
 * workgroup, so the wait always ends; past the bound the iteration fails with HMMBW_E_TIMEOUT (EM stops,
 * the sweep's statistics are not added) instead of reading alpha_hat that may not be there.  Default
 * 10000; 0 expires at once (tests the error path). */
#define HMMBW_OPT_WQ_TIMEOUT_MS 11
/* Wide E-step work queue (a workgroup per forward and per backward sweep of each 16-sequence tile, taken
 * in dispatch order, so the CUs' loads even out in sweeps instead of whole tiles): -1 (default) when the
 * tiles exceed 4 per CU, 1 whenever they exceed the CU count, 0 never.  The environment variable
 * HMMBW_WIDE_WQ=0/1 sets a new context's default.  Takes effect at once. */
#define HMMBW_OPT_WIDE_WQ 12
int hmmbw_set_option(hmmbw_ctx *ctx, int key, int64_t value);
/* The current value of an option above, or a read-only fact about the loaded observations' E-step launch:
 * HMMBW_INFO_WIDE_WQ_ACTIVE    1 if it runs on the wide work queue;
 * HMMBW_INFO_WAVES             active waves (small kernels: sequence-group waves; wide: tiles x NP/16);
 * HMMBW_INFO_WORKGROUPS        workgroups of the spread map (full + extra); with HMMBW_INFO_JOINED = 1
 *                              the launch itself is HMMBW_INFO_FULL_WORKGROUPS workgroups of twice
 *                              HMMBW_INFO_WAVES_PER_WORKGROUP waves (see HMMBW_INFO_JOINED);
 * HMMBW_INFO_WAVES_PER_WORKGROUP  waves per workgroup of the spread map;
 * HMMBW_INFO_FULL_WORKGROUPS   workgroups with every wave active (small kernels: the spread map puts the
 *                              waves past one per SIMD into workgroups of HMMBW_INFO_EXTRA_WAVES active waves
 *                              after these);
 * HMMBW_INFO_EXTRA_WAVES       active waves of each workgroup after the full ones;
 * HMMBW_INFO_PEER_CHUNKS       chunks of the peer all-reduce payload (each rank writes and polls one flag
 *                              per (rank, chunk) per iteration), 0 without a peer region;
 * HMMBW_INFO_JOINED            1 if the E-step runs the joined map (left-to-right): extra workgroup b's
 *                              waves run as waves 4.. of full workgroup b, one 8-wave workgroup per CU, so
 *                              HMMBW_INFO_FULL_WORKGROUPS workgroups are launched (HMMBW_JOIN=0 turns it off);
 * HMMBW_INFO_SPLIT_EXTRA       1 if the extra workgroups' idle waves run the lower backward half of their
 *                              sequence groups (dense split; HMMBW_SPLIT_EXTRA=0 turns it off).
 * (bench.py's roofline bounds price the busiest CU and SIMD from this map.) */
#define HMMBW_INFO_WIDE_WQ_ACTIVE 101
#define HMMBW_INFO_WAVES 102
#define HMMBW_INFO_WORKGROUPS 103
#define HMMBW_INFO_WAVES_PER_WORKGROUP 104
#define HMMBW_INFO_FULL_WORKGROUPS 105
#define HMMBW_INFO_EXTRA_WAVES 106
#define HMMBW_INFO_PEER_CHUNKS 107
#define HMMBW_INFO_JOINED 108
#define HMMBW_INFO_SPLIT_EXTRA 109
/* diagnostics: device address of the peer all-reduce's sum buffer (the pending M-step's source), 0 without
 * a peer region (tools/peer_diag.py) */
#define HMMBW_INFO_PEER_SUM_PTR 110
/* process-wide: uncached / fine-grained peer regions validated, and rejected (quarantined) because kernel
 * loads did not read back what was written (see hmmbw.hip, peer_region_alloc) */
#define HMMBW_INFO_PEER_REGIONS_VALIDATED 111
#define HMMBW_INFO_PEER_REGIONS_REJECTED 112
int hmmbw_get_option(const hmmbw_ctx *ctx, int key, int64_t *value);

/* E-step kernel timing with HIP events on the context stream (for bench/roofline).  Returns the
 * accumulated time and count of the timed launches so far, then (enable >= 0) resets and sets the
 * mode: 0 off, k >= 1 record events around every k-th E-step launch (sampling keeps the event
 * overhead out of the timed loop); enable < 0 only queries. */
int hmmbw_timing(hmmbw_ctx *ctx, int enable, double *total_ms, int64_t *count);
/* The timed launches that run a follow-up kernel after the E-step kernel (the wide path's B-numerator
 * gather, hmm_training.py:474-485; deterministic mode's fixed-order reductions): the accumulated time of
 * the E-step kernel alone and the count (same reset as hmmbw_timing).  bench.py prices the fp64-MFMA
 * bound on it. */
int hmmbw_timing_split(hmmbw_ctx *ctx, double *estep_ms, int64_t *count);

/* Vector-quantisation encoder: get_observations, hmm_training.py:82-120.  For every frame f, the index
 * of the nearest centroid (first minimum, strict '<' as at :111) by the Euclidean distance over the
 * columns [first_dim, first_dim + dims) of frames[f * frame_stride ...] and centroids[k * frame_stride
 * ...] (the reference: stride 13, first_dim 1 — mfcc[1:] without the power coefficient — dims 12),
 * computed exactly as np.linalg.norm does (sequential fused multiply-add, correctly rounded sqrt), so
 * the indices are bit-identical to the reference's.  DEVICE pointers (frames [n_frames][stride],
 * centroids [n_centroids][stride] fp64, symbols int32 [n_frames], distances fp64 [n_frames] or NULL:
 * the winning distance, the reference's min_distance); enqueued on `stream` (hipStream_t, NULL =
 * legacy default), asynchronous; the device is the current one.  Codebook <= 160 KiB. */
int hmmbw_vq_encode(void *stream, const double *frames, int64_t n_frames, int frame_stride, int first_dim, int dims,
                    const double *centroids, int n_centroids, int32_t *symbols, double *distances);

/* ---- Groups: several models of one shape, one launch per EM iteration / per scoring pass ----
 * The reference trains its word models one after another (train_hmm, HMM/main.py:147-152, calling
 * training_with_save -> hmm_training once per word, hmm_training.py:215-247) and scores every
 * (recording, model) pair with its own forward pass (test_hmm, HMM/hmm_testing.py:139-161).  A group
 * advances all member contexts with ONE grouped E-step launch per iteration (each member's M-step runs
 * in its slice's prologue; each member keeps its own parameters, statistics, convergence state and
 * stop rule, exactly as if trained alone) and scores all of them with one launch.
 * Members: single-rank contexts on the same device and stream, with equal N, M and resolved topology,
 * N <= 16 and emission tables that fit LDS, each with observations and parameters set (checked at
 * creation, HMMBW_E_UNSUPPORTED otherwise, and again at every call); the group does not own them
 * (destroy the group first). */
typedef struct hmmbw_group hmmbw_group;
int hmmbw_group_create(hmmbw_ctx *const *ctxs, int n, hmmbw_group **out);
int hmmbw_group_destroy(hmmbw_group *group);
/* hmmbw_iterate(ctx, n_iter) for every member (arm each with hmmbw_reset_training first). */
int hmmbw_group_iterate(hmmbw_group *group, int64_t n_iter);
/* SYNC. hmmbw_score of every member, concatenated in member order (sum of the members' R doubles). */
int hmmbw_group_score(hmmbw_group *group, double *out);
/* Timing of the grouped E-step launches (same protocol as hmmbw_timing). */
int hmmbw_group_timing(hmmbw_group *group, int enable, double *total_ms, int64_t *count);

#ifdef __cplusplus
}
#endif
#endif /* HMMBW_H */
