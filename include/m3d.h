/*
 * m3d.h — C ABI of the MI355X-native point-cloud registration core (libm3d.so, gfx950).
 *
 * Drop-in boundary for the hot path of KTC-Security-Circle/3d-matching `src/matcher`
 * (SURVEY.md §8(b)).  The reference has no FFI of its own: its "plugin API" is the Python
 * functions of `src/matcher/ransac.py` and `src/matcher/icp.py`, which call numpy and the
 * Open3D 0.19 C++ registration pipeline.  Each entry point below names the reference interface
 * it replaces; the Python mirror (3d-matching_amd/matcher) binds them through ctypes.
 *
 * Conventions
 *   - Plain C types only; no torch types.  Array arguments marked [device] are caller-owned
 *     device allocations (e.g. torch.cuda tensors' data_ptr()); [host] are host memory.
 *   - Point arrays are float64 AoS N×3 (24 B/pt), exactly the layout of Open3D's
 *     Vector3dVector / numpy (N,3) the reference uses; correspondences are int32 N×2.
 *   - 4×4 transforms are float64 row-major (numpy order).
 *   - `stream` is a hipStream_t (NULL = legacy default stream).  Every entry point only
 *     enqueues work on `stream` unless documented as synchronous (the *_run functions and the
 *     object constructors return host values and synchronise the stream).
 *   - Return value: M3D_OK (0) or a negative M3D_ERR_*; m3d_last_error(ctx) explains it.
 *     Numerical failure of a hypothesis is NOT an error: as in the reference
 *     (ransac.py:134-140,184-192) it yields the identity transform and a per-hypothesis status.
 *   - One context per (host thread, device).  A context owns its scratch memory; the library
 *     never frees caller memory.  Calls on one context that use its scratch (the RANSAC entry
 *     points) may pass different streams: a call on another stream than the previous one first
 *     waits on the device for the previous call's work (no host synchronisation), so such calls
 *     are ordered, not concurrent.
 */
#ifndef M3D_H_
#define M3D_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define M3D_ABI_VERSION 13

/* return codes */
#define M3D_OK 0
#define M3D_ERR_INVALID (-1)  /* bad argument (sizes, null pointers, missing normals, ...) */
#define M3D_ERR_HIP (-2)      /* HIP runtime error */
#define M3D_ERR_OOM (-3)      /* device allocation failed */
#define M3D_ERR_NODEVICE (-4) /* no usable gfx950 device */
#define M3D_ERR_COMM (-5)     /* a peer rank failed, or the communicator was aborted (ABI 8) */

/* per-hypothesis status (ransac.py:134-140,184-192) */
#define M3D_HYP_OK 0
#define M3D_HYP_DEGENERATE 1 /* fewer than 3 correspondences -> identity */
#define M3D_HYP_NONFINITE 2  /* NaN/Inf in the estimate -> identity */

/* inlier comparator */
#define M3D_SCORE_SQUARED 0 /* Σd² < thr   (evaluate_inlier_ratio_fast, ransac.py:274-277) */
#define M3D_SCORE_NORM 1    /* ‖d‖ < thr    (evaluate_inlier_ratio,      ransac.py:233-236) */

/* ICP estimators (Open3D TransformationEstimation*) */
#define M3D_EST_POINT_TO_POINT 0
#define M3D_EST_POINT_TO_PLANE 1

typedef struct m3d_ctx m3d_ctx;
typedef struct m3d_corrset m3d_corrset; /* packed correspondence set (RANSAC) */
typedef struct m3d_cloud m3d_cloud;     /* packed point cloud (ICP / NN)      */
typedef struct m3d_icp m3d_icp;         /* device-resident ICP loop state     */

/* ------------------------------------------------------------------ context */
int m3d_abi_version(void);
int m3d_device_count(int* count);
int m3d_create(int device, m3d_ctx** out);
void m3d_destroy(m3d_ctx* ctx);
const char* m3d_last_error(const m3d_ctx* ctx);
/* Device-side hit counters (cumulative): [0] pairs rechecked in fp64 by the scoring screens
 * (guard band), [1] by full hypothesis; the others are reserved (0). */
int m3d_get_stats(m3d_ctx* ctx, int64_t* out8 /* [host] 8 values */);

/* Kernel timing with HIP events recorded on the launch stream immediately before and after each
 * launch of the named kernel (benchmarks / roofline).  Kernel ids: */
#define M3D_KERNEL_NN 0     /* ICP brute-force NN scan          */
#define M3D_KERNEL_SCORE 1  /* RANSAC fp32 scoring screen       */
#define M3D_KERNEL_KABSCH 2 /* RANSAC batched 3-point Kabsch    */
#define M3D_KERNEL_TERMS 3  /* ICP fp64 estimation terms        */
#define M3D_KERNEL_LOOP 4   /* reserved (ABI 10-11: the persistent grid loop, removed in ABI 12) */
#define M3D_KERNEL_COMM 5   /* RCCL all-reduces issued by the library, on their streams (ABI 10) */
int m3d_profile_enable(m3d_ctx* ctx, int enable);
/* Synchronises, returns Σ launch durations (ms) and launch count since the last read, resets. */
int m3d_profile_read(m3d_ctx* ctx, int kernel, double* total_ms, int64_t* launches);

/* ------------------------------------------------------------------ RANSAC */

/* Gather + pack a correspondence set: p_i = src[corr[i,0]], q_i = tgt[corr[i,1]].
 * Replaces the per-call gathers of evaluate_inlier_ratio (ransac.py:223-227) and the
 * pre-gather of _visualize_matcher.py:376-384.  Synchronous (computes centring offsets).
 * src_xyz [device] ns×3 f64, tgt_xyz [device] nt×3 f64, corr [device] nc×2 int32. */
int m3d_corrset_create(m3d_ctx* ctx, const double* src_xyz, int64_t ns, const double* tgt_xyz,
                       int64_t nt, const int32_t* corr, int64_t nc, void* stream,
                       m3d_corrset** out);
/* Same from pre-gathered pairs (the p_src / p_tgt arguments of evaluate_inlier_ratio_fast,
 * ransac.py:239-244): p_src, p_tgt [device] nc×3 f64. */
int m3d_corrset_create_gathered(m3d_ctx* ctx, const double* p_src, const double* p_tgt,
                                int64_t nc, void* stream, m3d_corrset** out);
void m3d_corrset_destroy(m3d_corrset* cs);
int64_t m3d_corrset_size(const m3d_corrset* cs);

/* a1, batched: H hypotheses of compute_step_transformation (ransac.py:104-192).
 * triples [device] H×3 int32 correspondence rows (replay mode: e.g. the rows the reference's
 * np.random.choice(n,3,replace=False) draws, see m3d_replay_triples), or NULL for the native
 * counter-based sampler keyed by (seed, hyp0 + h).
 * T_out [device] H×16 f64 row-major; status [device] H uint8 (may be NULL). */
int m3d_kabsch3_batch(m3d_ctx* ctx, const m3d_corrset* cs, const int32_t* triples,
                      uint64_t seed, int64_t hyp0, int64_t H, double* T_out, uint8_t* status,
                      void* stream);

/* a2/a3, batched: counts[h] = #{i : dist(T_h p_i, q_i) < thr} for H transforms.
 * mode M3D_SCORE_SQUARED: thr is the squared threshold (evaluate_inlier_ratio_fast);
 * mode M3D_SCORE_NORM:    thr is the distance threshold (evaluate_inlier_ratio).
 * T [device] H×16 f64; counts [device] H int32.  Counts are exact w.r.t. an fp64 evaluation
 * of the reference formula (fp32 screen + fp64 recheck of pairs inside a proven guard band). */
int m3d_ransac_score(m3d_ctx* ctx, const m3d_corrset* cs, const double* T, int64_t H, double thr,
                     int mode, int32_t* counts, void* stream);

/* a1 and a2/a3 for ONE hypothesis with host operands — the per-call form the reference harness
 * uses (benchmark_ransac.py:105-113: one compute_step_transformation + one
 * evaluate_inlier_ratio per iteration).  Synchronous; the operands travel as kernel arguments
 * and the results come back through the context's mapped pinned memory (one launch + one
 * stream sync each; a2/a3 evaluates the reference formula directly in fp64, numpy's order).
 * m3d_kabsch3_one: triple [host] 3 int32 rows; T_out [host] 16 f64; status [host] (may be
 * NULL) M3D_HYP_*.  Replaces compute_step_transformation (ransac.py:104-192) after its
 * np.random.choice draw (ransac.py:143).
 * m3d_ransac_score_one: T [host] 16 f64; *count [host] = inliers (thr / mode as in
 * m3d_ransac_score).  Replaces evaluate_inlier_ratio[_fast] (ransac.py:195-277). */
int m3d_kabsch3_one(m3d_ctx* ctx, const m3d_corrset* cs, const int32_t* triple, double* T_out,
                    int32_t* status, void* stream);
int m3d_ransac_score_one(m3d_ctx* ctx, const m3d_corrset* cs, const double* T, double thr,
                         int mode, int64_t* count, void* stream);

/* a4: the step-RANSAC loop (_visualize_matcher.py:343-470; benchmark_ransac.py:87-125 when
 * early_stop == 0), run on the device in batches with no host round trip per batch. */
typedef struct {
  int64_t max_iter;     /* MatcherSettings.ransac_iteration                          */
  uint64_t seed;        /* native sampler seed (ignored when triples are supplied)   */
  double thr;           /* comparator threshold (see mode)                           */
  int32_t mode;         /* M3D_SCORE_SQUARED (GUI loop, a3) or M3D_SCORE_NORM (a2)   */
  int32_t early_stop;   /* MatcherSettings.early_stop_enabled                        */
  double es_threshold;  /* MatcherSettings.early_stop_threshold (0.5)                */
  double es_confidence; /* MatcherSettings.early_stop_confidence (0.99)              */
  int64_t batch;        /* hypotheses per device batch (0 = automatic)               */
  int64_t hyp0;         /* first hypothesis id (multi-GPU hypothesis sharding)       */
} m3d_ransac_params;

typedef struct {
  double T[16];        /* best transform (row-major)                        */
  double fitness;      /* best inlier ratio = best_count / nc                */
  int64_t best_index;  /* 0-based iteration index of the best hypothesis     */
  int64_t iterations;  /* iter_num at exit (early stop or max_iter)          */
  int64_t best_count;  /* inlier count of the best hypothesis                */
  int64_t rechecked;   /* pairs re-evaluated in fp64 (guard band)            */
} m3d_ransac_result;

/* triples [device] max_iter×3 int32 or NULL (native sampler).  Synchronous. */
int m3d_ransac_run(m3d_ctx* ctx, const m3d_corrset* cs, const m3d_ransac_params* params,
                   const int32_t* triples, m3d_ransac_result* out, void* stream);
/* Asynchronous form: per-hypothesis counts of the whole run land in counts_out [device]
 * (max_iter int32, may be NULL; hypotheses after an early stop are not scored and read 0) and
 * the result struct in result_dev [device]. */
int m3d_ransac_run_async(m3d_ctx* ctx, const m3d_corrset* cs, const m3d_ransac_params* params,
                         const int32_t* triples, int32_t* counts_out, m3d_ransac_result* result_dev,
                         void* stream);

/* Host-side replay of the reference RNG: the rows H successive
 * `np.random.choice(nc, 3, replace=False)` calls of the legacy MT19937 RandomState draw
 * (ransac.py:143 ≡ permutation(nc)[:3]).  mt_key [host] 624 uint32 + *mt_pos is the state
 * `np.random.get_state()` returns; both are advanced in place exactly as numpy would.
 * triples_out [host] H×3 int32. */
int m3d_replay_triples(uint32_t* mt_key, int32_t* mt_pos, int64_t nc, int64_t H,
                       int32_t* triples_out);

/* ------------------------------------------------------------------ ICP */

/* Pack a cloud for NN / ICP: xyz [device] n×3 f64, normals [device] n×3 f64 or NULL.
 * Synchronous (computes the centring offset).  Replaces Open3D's PointCloud copy +
 * KDTreeFlann::SetGeometry (Registration.cpp RegistrationICP). */
int m3d_cloud_create(m3d_ctx* ctx, const double* xyz, const double* normals, int64_t n,
                     void* stream, m3d_cloud** out);
/* The same with an explicit centring offset center [host] 3 f64 instead of the cloud's mean.
 * Shards of one target cloud created with the same centre share one fp32 frame, so their NN
 * keys are comparable bit for bit: target-sharded ICP (m3d_icp_shard_nn on each rank, MIN of
 * the keys) then seeds the queries whose previous winner another rank owns with a distance
 * bound instead of the radius (nnkey.h seed_key) — same result, far fewer screen hits. */
int m3d_cloud_create_framed(m3d_ctx* ctx, const double* xyz, const double* normals, int64_t n,
                            const double* center, void* stream, m3d_cloud** out);
/* The same from HOST arrays (ABI 11): xyz [host] n×3 f64, normals [host] n×3 f64 or NULL, center
 * [host] 3 f64 or NULL (the cloud's mean).  The arrays go straight into the cloud's buffers
 * (one pageable copy each) instead of a caller's upload plus a device-to-device copy.  The same
 * cloud, bit for bit.  Synchronous. */
int m3d_cloud_create_host(m3d_ctx* ctx, const double* xyz, const double* normals, int64_t n,
                          const double* center, void* stream, m3d_cloud** out);
/* Destroy a cloud.  Its device blocks go to the library's block cache, marked after all work
 * its context had enqueued on any stream; a later allocation reuses them in stream order (the
 * allocating stream waits on the device; no host or device-wide synchronisation, ABI 12).
 * An m3d_icp created on this cloud may outlive it: the loop keeps the data it runs on and frees
 * it in m3d_icp_destroy (ABI 12); stepping a loop whose TARGET cloud is gone is undefined.
 * Destroy every object before its context. */
void m3d_cloud_destroy(m3d_cloud* c);
int64_t m3d_cloud_size(const m3d_cloud* c);
/* Give the block cache's idle blocks of ctx's device back to the driver (each after its release
 * point has passed on the device); freed_bytes may be NULL.  The Python layer calls this when a
 * device allocation fails; the library does so itself before retrying its own allocations, and
 * when the last context of a device is destroyed.  M3D_BLOCK_CACHE=<MiB> caps the cache (default
 * 2048, 0 = no cache).  ABI 12. */
int m3d_trim_block_cache(m3d_ctx* ctx, int64_t* freed_bytes);

/* Nearest-neighbour search method.  Both return the identical (d², index) result: BRUTE scans
 * every target (cfg1's LDS-tiled brute force), GRID visits only the uniform-grid cells that can
 * hold a target within the radius. */
#define M3D_NN_BRUTE 0
#define M3D_NN_GRID 1

/* Radius-bounded 1-NN (KDTreeFlann::SearchHybrid(p, r, 1) for every source point after T):
 * idx [device] ns int32 (-1 = no target with d² < r²), d2 [device] ns f64 (may be NULL). */
int m3d_nn1(m3d_ctx* ctx, const m3d_cloud* src, const m3d_cloud* tgt, const double* T_host,
            double max_dist, int32_t nn_method, int32_t* idx, double* d2, void* stream);

typedef struct {
  double relative_fitness; /* ICPConvergenceCriteria defaults 1e-6 */
  double relative_rmse;    /* 1e-6 */
  int32_t max_iteration;   /* 30 */
  int32_t estimation;      /* M3D_EST_* */
  int32_t nn_method;       /* M3D_NN_* */
  int32_t flags;           /* M3D_ICP_* (ABI 10; 0 = defaults) */
} m3d_icp_params;
/* m3d_icp_params.flags 1 and 4 (ABI 10-11: the persistent grid loop on / off) are accepted and
 * ignored since ABI 12, which removed that loop (measured slower than the two-launch steps). */
#define M3D_ICP_NO_PERSIST 1
#define M3D_ICP_PERSIST 4
/* m3d_icp_params.flags: the target-shard loop exchanges all keys in one MIN instead of two halves
 * overlapped with the second half's NN (m3d_icp_shard_steps) */
#define M3D_ICP_NO_SPLIT 2

typedef struct {
  double T[16];
  double fitness;
  double inlier_rmse;
  int64_t num_correspondences;
  int32_t iterations; /* updates applied */
  int32_t converged;
  double update[16];  /* the last update ΔT (identity after a reset), ABI 12 */
} m3d_icp_result;

/* registration_icp (icp.py:42-48 → Open3D RegistrationICP).  init [host] 16 f64.
 * corr_idx [device] ns int32 or NULL: final correspondence target per source (-1 = none).
 * Synchronous. */
int m3d_icp_run(m3d_ctx* ctx, const m3d_cloud* src, const m3d_cloud* tgt, const double* init,
                double max_dist, const m3d_icp_params* params, m3d_icp_result* out,
                int32_t* corr_idx, void* stream);

/* Step-wise ICP driver (benchmarks, multi-GPU).  An m3d_icp holds the device-resident loop
 * state (T, fitness/rmse history, convergence flag); every call only enqueues work. */
int m3d_icp_create(m3d_ctx* ctx, const m3d_cloud* src, const m3d_cloud* tgt, double max_dist,
                   const m3d_icp_params* params, m3d_icp** out);
void m3d_icp_destroy(m3d_icp* s);
/* init [host] 16 f64 or NULL (identity).  As RegistrationICP (Registration.cpp): T starts at
 * init, and the loop's copy of the source is transformed by init only when init is not
 * Eigen-isIdentity() (|a − δ| ≤ 1e-12); every update ΔT then transforms that copy again
 * (pcd.Transform(update)), and each evaluation's fp64 queries are those points (ABI 12: before,
 * the queries were T·p of the original source). */
int m3d_icp_reset(m3d_icp* s, const double* init_host, void* stream);
/* The loop's fp64 points of the last evaluation (the source after init and every update but the
 * one the evaluation produced), dst [device] ns×3 f64 in the caller's source order.  After a reset
 * and before the first evaluation: the source with the init applied exactly as RegistrationICP's
 * pcd.Transform(init) (the source itself when init isIdentity()).  ABI 12; init applied ABI 13. */
int m3d_icp_copy_points(const m3d_icp* s, double* dst, void* stream);
/* One full iteration on one device: NN evaluation + estimation terms + solve/update. */
int m3d_icp_step(m3d_icp* s, void* stream);
/* n iterations (n × m3d_icp_step, enqueued from native code: no per-iteration host binding
 * overhead).  Iterations after convergence / max_iteration are device no-ops.  A sequence of n
 * steps requested a second time (from the same keys state) is captured into a HIP graph and
 * replayed as one launch from then on (M3D_ICP_GRAPH=0: plain enqueues); the results are the
 * same bits either way. */
int m3d_icp_steps(m3d_icp* s, int32_t n, void* stream);
/* Capture the n-step graph now, for the loop's current state (setup work, e.g. before a timed
 * region; nothing runs).  Later m3d_icp_steps(s, n) calls from that state replay it. */
int m3d_icp_prepare_steps(m3d_icp* s, int32_t n);
/* Multi-GPU pieces (icp.py:42-48 with the correspondence search split over ranks).
 * Result contract of every NN (nnkey.h): for each source point the lexicographic (d64, index)
 * minimum over the targets with d64 < r², d64 the fp64 d² of the fp64 transformed point —
 * identical on one device and over any number of target shards.
 *
 * Target shard (cfg3): `tgt` of m3d_icp_create is this rank's shard whose first point has global
 * index shard_offset (create every shard with the same centre, m3d_cloud_create_framed).  Per
 * iteration, with the exchanges done by the caller (or m3d_comm_*):
 *   m3d_icp_shard_nn(s, off, dkeys)      this shard's fp64 winners; dkeys [device] ns int64 =
 *                                        bits(d64) (INT64_MAX none)          → all-reduce MIN
 *   m3d_icp_shard_claim(s, dmin, claim)  claim [device] ns int32 = own target index where the own
 *                                        winner has the global d64, else INT32_MAX → all-reduce MIN
 *                                        (exact fp64 ties across shards → lowest index)
 *   m3d_icp_shard_terms(s, off, dmin, claim, sums)  terms of the owned winners; sums [device]
 *                                        32 f64                               → all-reduce SUM
 *   m3d_icp_solve(s, sums)               identical update on every rank.
 * Every per-source exchange buffer (dkeys, dmin, claim) is indexed by the loop's SOURCE SLOT: the
 * loop keeps its source in the Morton order of the source's grid (coalesced per-source arrays);
 * m3d_icp_copy_slots gives slot → source index.  Ranks that share one source cloud (the target
 * shard) get the same slots.
 * Source shard (SURVEY §8(e) "ICP alternative"): `src` is this rank's source shard, `tgt` the
 * whole target: m3d_icp_shard_nn(s, 0, NULL) + m3d_icp_shard_terms(s, 0, NULL, NULL, sums),
 * SUM of the sums, m3d_icp_solve; the fitness denominator is m3d_icp_set_source_total's. */
int m3d_icp_shard_nn(m3d_icp* s, int64_t shard_offset, int64_t* dkeys, void* stream);
/* m3d_icp_shard_nn for the source slots [q0, q1) only (dkeys entries outside stay untouched): the
 * pieces of the split exchange (ABI 8).  M3D_ERR_INVALID when the loop's NN has no range form. */
int m3d_icp_shard_nn_range(m3d_icp* s, int64_t shard_offset, int64_t q0, int64_t q1, int64_t* dkeys,
                           void* stream);
int m3d_icp_shard_claim(m3d_icp* s, const int64_t* dmin, int32_t* claim, void* stream);
int m3d_icp_shard_terms(m3d_icp* s, int64_t shard_offset, const int64_t* dmin, const int32_t* claim,
                        double* sums, void* stream);
int m3d_icp_solve(m3d_icp* s, const double* sums, void* stream);
/* Source-sharded runs: the source count over all ranks (0 = this shard's own count). */
int m3d_icp_set_source_total(m3d_icp* s, int64_t ns_total);
/* ------------------------------------------------------------------ RCCL inside the library
 * (SURVEY §8(b)/(e)): one communicator per (context, rank) over RCCL/xGMI; the caller only
 * carries the 128-byte unique id from rank 0 to the others (e.g. torch.distributed's
 * broadcast_object_list) — the collectives of the multi-GPU loops are issued by libm3d on the
 * caller's stream, with no host round trip. */
typedef struct m3d_comm m3d_comm;
#define M3D_COMM_ID_BYTES 128
#define M3D_DT_I32 0
#define M3D_DT_I64 1
#define M3D_DT_F64 2
#define M3D_OP_SUM 0
#define M3D_OP_MIN 1
#define M3D_OP_MAX 2
/* id_out [host] M3D_COMM_ID_BYTES bytes (ncclGetUniqueId), called on rank 0. */
int m3d_comm_unique_id(uint8_t* id_out);
/* Collective over the world's ranks (every rank calls it with the same id).  Synchronous.  Every
 * buffer the library's collectives use is allocated here or before a loop's first collective.
 * Failure contract (ABI 8): a loop object's first multi-GPU call allocates its exchange buffers
 * and all ranks agree on the outcome (a rank whose setup failed returns its error, its peers
 * M3D_ERR_COMM — nobody enters the loop); m3d_ransac_run_sharded is fail-soft (a failed local run
 * still joins the collectives, every rank returns an error); a launch or RCCL error inside a
 * collective loop aborts the communicator (ncclCommAbort) and every later call on it returns
 * M3D_ERR_COMM — peers already waiting in a collective cannot be reached from that rank, so the
 * caller must then tear down every rank (torch.distributed.run does when a worker fails). */
int m3d_comm_init(m3d_ctx* ctx, const uint8_t* id, int rank, int world, m3d_comm** out);
void m3d_comm_destroy(m3d_comm* c);
/* In-place all-reduce of buf [device] count elements of dtype M3D_DT_* with op M3D_OP_*. */
int m3d_comm_allreduce(m3d_comm* c, void* buf, int64_t count, int dtype, int op, void* stream);
/* n iterations of target-sharded ICP (the protocol of "Multi-GPU pieces" above) with the MIN /
 * MIN / SUM all-reduces issued inside; every rank calls it with its shard offset.  The sources
 * are split into two slot halves: the first half's d64 MIN runs on a library-owned exchange
 * stream while the second half's NN runs on `stream` (M3D_SHARD_SPLIT=0: one piece). */
int m3d_icp_shard_steps(m3d_icp* s, m3d_comm* c, int64_t shard_offset, int32_t n, void* stream);
/* n iterations of source-sharded ICP (one SUM of the 32 term slots per iteration). */
int m3d_icp_source_shard_steps(m3d_icp* s, m3d_comm* c, int32_t n, void* stream);
/* Hypothesis-sharded a4 without early stop (cfg2 at N > 1): after m3d_ransac_run_async on each
 * rank's id range [hyp0, hyp0 + max_iter), key_dev [device] 1 int64 ← MAX over ranks of
 * (best_count << 32) | (2³² − 1 − (hyp0 + best_index)): highest count, lowest global id. */
int m3d_ransac_best_allreduce(m3d_comm* c, const m3d_ransac_result* result_dev, int64_t hyp0,
                              int64_t* key_dev, void* stream);
/* The whole hypothesis-sharded run, synchronous (one host sync): out holds the global winner
 * (its transform's bits from the winning rank via an integer SUM; best_index = global id;
 * iterations and rechecked summed over ranks).  params->early_stop must be 0 and the native
 * sampler is used.  Scratch is the communicator's (no allocation per call). */
int m3d_ransac_run_sharded(m3d_ctx* ctx, m3d_comm* c, const m3d_corrset* cs,
                           const m3d_ransac_params* params, m3d_ransac_result* out, void* stream);
/* 1 once the communicator was aborted after a failure (M3D_ERR_COMM from then on), else 0. */
int m3d_comm_poisoned(const m3d_comm* c);

/* Read the loop state (synchronises the stream).  M3D_ERR_HIP when the grid NN's deferral list
 * overflowed since the last reset (its writes were dropped, the keys are not valid; ABI 13). */
int m3d_icp_result_get(m3d_icp* s, m3d_icp_result* out, void* stream);
/* The correspondence set of a per-source index array (RegistrationResult.correspondence_set,
 * icp.py:42 / ransac.py:42-59; ABI 11): pairs_out [host] with room for 2·n int32 receives
 * (i, corr_idx[i]) for every i with corr_idx[i] >= 0, in increasing i; *count [host] = the number
 * of pairs.  corr_idx [device] n int32 (m3d_icp_run's corr_idx, m3d_icp_copy_corr's dst, the
 * feature RANSAC's corr_set_out).  Compacted on the device; only the pairs cross to the host.
 * Synchronous. */
int m3d_corr_pairs(m3d_ctx* ctx, const int32_t* corr_idx, int64_t n, int32_t* pairs_out, int64_t* count,
                   void* stream);
/* Device pointer to the current correspondence index array (ns int32, -1 = none) in SOURCE SLOT
 * order (see m3d_icp_copy_slots); m3d_icp_copy_corr gives it in source order. */
const int32_t* m3d_icp_corr(const m3d_icp* s);
/* Copy the current correspondence array to dst [device] (ns int32, source order: dst[i] = target
 * index of source point i, -1 = none). */
int m3d_icp_copy_corr(const m3d_icp* s, int32_t* dst, void* stream);
/* dst [device] ns int32: dst[k] = the source point index held in slot k (ABI 8). */
int m3d_icp_copy_slots(const m3d_icp* s, int32_t* dst, void* stream);

/* ------------------------------------------------------------------ preprocessing
 * Open3D 0.19 semantics restated (oracle/prep_oracle.py); all fp64. */

/* PointCloud::VoxelDownSample (src/ply/ply.py:106).  xyz [device] n×3, normals [device] n×3 or
 * NULL; out_xyz / out_normals [device] with room for n×3; *out_n [host] = voxels.  Voxels come in
 * ascending (ix, iy, iz) order (Open3D: unordered_map order, unspecified).  Synchronous. */
int m3d_voxel_down_sample(m3d_ctx* ctx, const double* xyz, const double* normals, int64_t n,
                          double voxel_size, double* out_xyz, double* out_normals, int64_t* out_n,
                          void* stream);
/* KDTreeFlann::SearchHybrid(p_i, radius, max_nn) for every point of the cloud (strict d² < r²,
 * ascending (d², index)).  idx [device] n×max_nn int32 (-1 pad), d2 [device] n×max_nn f64,
 * count [device] n int32.  Synchronous. */
int m3d_hybrid_search(m3d_ctx* ctx, const m3d_cloud* cloud, double radius, int32_t max_nn,
                      int32_t* idx, double* d2, int32_t* count, void* stream);
/* PointCloud::EstimateNormals(KDTreeSearchParamHybrid(radius, max_nn)) (ply.py:110-112,133-135):
 * covariance of the hybrid neighbourhood → FastEigen3x3; the cloud's own normals, if any, orient
 * the result.  normals_out [device] n×3.  Synchronous. */
int m3d_estimate_normals(m3d_ctx* ctx, const m3d_cloud* cloud, double radius, int32_t max_nn,
                         double* normals_out, void* stream);
/* ComputeFPFHFeature(cloud, KDTreeSearchParamHybrid(radius, max_nn)) (ply.py:117-120).
 * normals [device] n×3; fpfh_out [device] n×33 row-major (Open3D's Feature.data is 33×n).
 * Synchronous. */
int m3d_compute_fpfh(m3d_ctx* ctx, const m3d_cloud* cloud, const double* normals, double radius,
                     int32_t max_nn, double* fpfh_out, void* stream);

/* ------------------------------------------------------------------ feature matching (a5, a6) */

/* CorrespondencesFromFeatures (src/matcher/ransac.py:85): exact fp64 1-NN in feature space
 * (lowest index on ties), optional mutual filter with Open3D's fallback to the one-directional
 * set below mutual_consistent_ratio·ns pairs.  f_src [device] ns×dim, f_tgt [device] nt×dim
 * (dim = 33), corr_out [device] room for ns×2 int32, *n_out [host].  Synchronous. */
int m3d_feature_correspondences(m3d_ctx* ctx, const double* f_src, int64_t ns, const double* f_tgt,
                                int64_t nt, int32_t dim, int32_t mutual_filter,
                                double mutual_consistent_ratio, int32_t* corr_out, int64_t* n_out,
                                void* stream);

typedef struct {
  double max_correspondence_distance; /* ransac.py:41 1.5·v */
  double confidence;                  /* RANSACConvergenceCriteria.confidence (0.999) */
  double edge_length;                 /* CorrespondenceCheckerBasedOnEdgeLength (0.9); <= 0 off */
  double distance;                    /* CorrespondenceCheckerBasedOnDistance (1.5·v); <= 0 off */
  uint64_t seed;                      /* counter sampler seed */
  int32_t max_iteration;              /* RANSACConvergenceCriteria.max_iteration (30) */
  int32_t ransac_n;                   /* 3 (only value supported; < 3 → empty result) */
} m3d_feature_ransac_params;

typedef struct {
  double T[16];
  double fitness;
  double inlier_rmse;
  int64_t best_index;  /* hypothesis id of the best, -1 = none */
  int64_t validations; /* hypotheses that passed the checkers and were validated */
  double corres_ratio; /* the best's correspondence inlier ratio (the exit estimate's input; ABI 10) */
} m3d_feature_ransac_result;

/* RegistrationRANSACBasedOnCorrespondence (ransac.py:44-58 → Open3D): PointToPoint (no scaling),
 * rows drawn with replacement by the counter sampler, checkers, validation over all source
 * points (1-NN within max_correspondence_distance), IsBetterRANSACThan, early exit as Open3D
 * 0.19: after each new best k = ceil(log(1-c)/log(1-ratio^3)) with ratio = the share of the nc
 * input correspondences within max_correspondence_distance under that best (Registration.cpp
 * EvaluateInlierCorrespondenceRatio; ABI 10 — ABI ≤ 9 used the fitness).
 * corr [device] nc×2 int32 (source, target) rows.
 * corr_set_out [device] ns int32 or NULL: the best transform's correspondence per source point
 * (-1 none).  Synchronous. */
int m3d_ransac_on_correspondences(m3d_ctx* ctx, const m3d_cloud* src, const m3d_cloud* tgt,
                                  const int32_t* corr, int64_t nc,
                                  const m3d_feature_ransac_params* params,
                                  m3d_feature_ransac_result* out, int32_t* corr_set_out,
                                  void* stream);

/* ------------------------------------------------------------------ test hooks
 * Host-compiled copy of the device 3×3 linear algebra (same source), for CPU-side unit tests
 * of the math.  Never used by the product path. */
int m3d_debug_kabsch3_host(const double* src9, const double* tgt9, double* T16);
int m3d_debug_ldlt6_host(const double* A36, const double* b6, double* x6);  // the device solve's
                                                                       // rule: unpivoted, pivoted fallback
/* XXH64 of [p, p + len) (the chunk hash of m3d_content_keys; known-answer tests). */
uint64_t m3d_debug_xxh64(const void* p, size_t len, uint64_t seed);
/* XXH3-128 (default secret, seed 0) of [p, p + len), len >= 241 (the long-input path the content
 * keys use; known-answer tests against the xxhash package): out2 = (low, high). */
int m3d_debug_xxh3_128(const void* p, size_t len, uint64_t* out2);
/* Failure injection for the multi-GPU failure tests: what = 1 fails this rank's next local run of
 * m3d_ransac_run_sharded, 2 its next ICP shard-loop iteration (0 clears). */
int m3d_debug_comm_inject(m3d_comm* c, int what);
/* The FPFH swap test's correctly rounded acos (ddmath.h acos_cr, host-compiled copy of the device
 * code): out[k] = acos(u[k]) rounded to nearest, for the CPU test against mpmath.  ABI 13. */
int m3d_debug_acos_cr(const double* u, int64_t n, double* out);
/* The same on the device: out[k] [device] = acos_cr(u[k]) (mode 0) or the device libm's acos
 * (mode 1) for u [device] n f64.  ABI 13. */
int m3d_debug_acos_device(m3d_ctx* ctx, const double* u, int64_t n, double* out, int mode, void* stream);
/* Fill every idle block of the block cache on the current device with `byte` (synchronous); a
 * later object that reuses one starts from those bytes.  Returns the blocks filled (>= 0).  ABI 13. */
int m3d_debug_block_cache_fill(int byte);
/* Overwrite the count of a grid loop's deferral list (synchronous on stream): a count past the
 * list makes the next scan drop its writes and m3d_icp_result_get fail with M3D_ERR_HIP until the
 * next m3d_icp_reset.  M3D_ERR_INVALID when the loop defers nothing.  ABI 13. */
int m3d_debug_icp_defer_count(m3d_icp* s, uint32_t count, void* stream);

/* ------------------------------------------------------------------ host text I/O (§8(f) rank 4) */

/* ASCII number blocks of PLY files (m3d.plyio; replaces the C++ readers/writers the reference
 * calls: o3d.io.read_point_cloud, src/ply/ply.py:80, and trimesh's ASCII PLY export,
 * convert_stl-ply.py:1-11).  Host only, no device needed.
 * m3d_parse_ascii_rows: `rows` non-blank lines of exactly `cols` numbers from buf[0, len) →
 * out [host] rows×cols f64 (correctly rounded, as numpy's parser); *consumed = bytes used.
 * M3D_ERR_INVALID on anything else (short file, extra or non-numeric tokens).
 * m3d_format_ascii_rows: rows×cols f64 → text, one row per line, each number the shortest
 * representation that reads back to the same double; cap ≥ 32·rows·cols. */
int m3d_parse_ascii_rows(const char* buf, size_t len, int64_t rows, int32_t cols, double* out,
                         size_t* consumed);
int m3d_format_ascii_rows(const double* data, int64_t rows, int32_t cols, char* out, size_t cap,
                          size_t* written);
/* STL corner merge (convert_stl-ply.py:3-6, trimesh.load_mesh): xyz [host] n×3 f64 corners →
 * uniq [host] (≤ n)×3 f64 unique vertices in first-occurrence order (exact equality, -0.0 ≡ +0.0),
 * inverse [host] n int32 (corner → vertex id), *n_unique. */
int m3d_merge_vertices(const double* xyz, int64_t n, double* uniq, int32_t* inverse,
                       int64_t* n_unique);
/* Content keys of the drop-in's cache (m3d.cache): keys [host] 2·n uint64 (low, high), the
 * 128-bit key of each buffer [host] bufs[i], lens[i] bytes — its 64 KB chunks hashed with
 * XXH3-128 by a persistent host thread pool (a tail under 241 bytes joins the previous chunk),
 * then XXH3-128 of (chunk digests ‖ length ‖ chunk count) (ABI 10; ABI ≤ 9 chained 64-bit XXH64
 * chunk digests).  Non-cryptographic: unrelated contents collide with probability ≈ 2⁻¹²⁸.  The
 * same bytes give the same key whatever the thread count. */
int m3d_content_keys(const void* const* bufs, const size_t* lens, int32_t n, uint64_t* keys);

#ifdef __cplusplus
}
#endif
#endif /* M3D_H_ */
