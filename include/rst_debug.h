/*
 * rst_debug.h -- diagnostics of the MI355X ICP library (not part of the
 * drop-in boundary; used by scripts/ and tests/ to explain performance).
 */
#ifndef RST_DEBUG_H_
#define RST_DEBUG_H_

#include "rst_align.h"

#ifdef __cplusplus
extern "C" {
#endif

/* rst_target_query_nn_warm plus per-wavefront search statistics: stats
 * receives 8 int32 per 64 queries (staging rounds, nodes tested, leaves
 * staged, leaves scanned, flushes, active lanes, lanes without a finite
 * starting bound, region extent in micrometres). */
int rst_debug_query_nn_warm_stats(rst_ctx* ctx, const rst_target* tgt, const float* q,
                                  int64_t nq, const int32_t* warm, int32_t* idx, float* d2,
                                  int32_t* stats);

/* Per iteration of the last align call on ctx (first n <= 256), 5 int32:
 * fallback-queue length (queries the level-1 adjacency could not certify),
 * queries answered by their candidate list (no search), unused, then the
 * solve kernel's reduction and solve times (10 ns ticks). */
int rst_debug_queue_trace(rst_ctx* ctx, int32_t* out, int32_t n);

/* RST_SUM_REF in-loop trace: with enable != 0, later aligns on ctx walk the
 * cost chain every iteration (not only the last, the only one the
 * reference reads, align_icp.cpp:104,157), and rst_debug_seq_trace gives, per
 * iteration of the last align (first n <= 256), 4 floats: the sequential
 * fp32 sums of the correspondences' x, y, z (dst_mean before the division,
 * :113) and of their d2 (the cost, :120) -- bit for bit the reference's
 * when every iteration's correspondences are. */
int rst_debug_enable_seq_trace(rst_ctx* ctx, int enable);
/* With the trace enabled, per iteration of the last align (first n <= 256)
 * the walks' statistics, 64 int32 each (the layout of rst_debug_seq_sum's
 * stats: per chain superblock tries / hits, group tries / hits, leaf tries
 * / hits, serial blocks, walker clocks; zero for chains of <= 16,384
 * elements, which k_sq_serial / k_sq_small sum without walk statistics). */
int rst_debug_seq_walk_stats(rst_ctx* ctx, int32_t* out, int32_t n);
/* Test hook: every sequential-sum walk after this call ORs `bits` (1..127,
 * 0 = off; process-wide) into its table bound-check word, as a corrupted map
 * would.  An align whose sums tripped a check returns RST_E_HIP (with
 * rst_last_error's detail), never the reference's false. */
int rst_debug_seqsum_fault(rst_ctx* ctx, int32_t bits);
/* The sequential sums' DPP scans (seqsum.hip wave_scan_incl /
 * block_scan_excl, the fp64 prefixes the maps' guesses come from) on one
 * wave: in[0..64) -> out[0..64) inclusive scan; in[64..128) -> out[64..128)
 * exclusive scan, out[128] the total. */
int rst_debug_wave_scan(rst_ctx* ctx, const double* in, double* out);
/* The context's reduction slab (first n doubles) as the last align left
 * it: diagnostics builds write kernel clocks there (tools/nn_clock.py). */
int rst_debug_slab(rst_ctx* ctx, double* out, int64_t n);
int rst_debug_seq_trace(rst_ctx* ctx, float* out, int32_t n);
/* The same for pair `pair` of the context's last collected batch
 * (rst_icp_align_batch_wait): per iteration its three dst sums; the cost
 * (column 3) only in the last iteration, where the batched loop walks it. */
int rst_debug_batch_seq_trace(rst_ctx* ctx, int32_t pair, float* out, int32_t n);

/* RST_DIAG builds, per iteration of the last align call on ctx (first n <=
 * 256), 4 int32: far-queue length, ball-tile chunks scanned (all waves),
 * ball-tile walks abandoned, deep (whole-wave) searches.  Zeros otherwise. */
int rst_debug_iter_diag(rst_ctx* ctx, int32_t* out, int32_t n);

/* The ICP loop's fallback search (one wavefront per query) on a host batch:
 * mode 0 = full walk from the warm leaf, 2 / 3 = level-2 / level-3
 * adjacency first, 23 = both then the walk.  warm = original target indices
 * (may be NULL); path[i] & 15 = 2, 3 or 0 (which strategy answered),
 * path[i] >> 4 = the search's shader cycles / 16.  Results equal
 * rst_target_query_nn's.  mode 1000: the ICP loop's two-nearest search
 * (level 2, level 3, walk; seeded with the warm point and its sorted
 * neighbour): idx/d2 as above, path[i] = the float bits of the
 * second-nearest d2 (FLT_MAX when m == 1). */
int rst_debug_query_nn_fallback(rst_ctx* ctx, const rst_target* tgt, const float* q,
                                int64_t nq, const int32_t* warm, int mode, int32_t* idx,
                                float* d2, int32_t* path);

/* The RST_SUM_REF loop's sequential sums on a host stream of n
 * float4: out[c] = ((0 + x[0].c) + x[1].c) + ... in float32, i ascending --
 * the rounding of `dst_mean += dst.GetPoint(j)` (align_icp.cpp:120). */
int rst_debug_seq_sum4(rst_ctx* ctx, const float* xyzw, int64_t n, float out[4]);

/* The same sums by either kernel: serial = 0 the loop's own choice by size
 * (seqsum_enqueue: the one-wavefront replay k_sq_serial up to
 * RST_SQ_SERIAL_MAX elements, the one-workgroup-per-component k_sq_small up
 * to RST_SQ_SMALL_MAX (<= 16384), else the parallel exact path -- verified
 * block / group / superblock maps, one walking wavefront per component),
 * 1 the older one-wavefront dependent chain (k_seq_sum4), 2 the map path
 * at any size, 3 k_sq_serial at any size, 4 k_sq_small up to 16384
 * elements (the map path beyond); reps launches back to back, *ms
 * (optional) = device time per launch; stats (optional, map path, 64
 * int32; untouched when k_sq_serial or the unforced k_sq_small ran; with
 * serial = 4, k_sq_small's own layout: [0..5] chain 0's phase clocks,
 * [8..13] group / leaf tries and hits, serial blocks, groups) = 8 per component
 * of the last launch's walk: superblock tries / hits, group tries / hits,
 * block tries / hits, blocks added serially, walker clocks; stats[32] =
 * the map kernels' bound-check failure bits (0 = none); stats[33 + c] =
 * component c's walker clocks waiting for superblock maps; stats[40 + 4c
 * + j] = its walker clock at the start of chunk j < 4 (16 superblocks a
 * chunk). */
int rst_debug_seq_sum(rst_ctx* ctx, const float* xyzw, int64_t n, int serial, int reps,
                      float out[4], float* ms, int32_t* stats);

/* The sequential sums' kernels one at a time (stages: bit 0 the front
 * kernel, bit 1 the maps, bit 2 the walk), each synchronised and checked
 * before the next is launched; the workspace (rst_debug_seq_ws_bytes(n)
 * bytes, zeroed first) is copied to ws_out (optional) afterwards, and
 * *failed_stage names the first kernel that failed (0 = none). */
int rst_debug_seq_stages(rst_ctx* ctx, const float* xyzw, int64_t n, int nch, int stages,
                         float out[4], void* ws_out, int64_t ws_bytes, int* failed_stage);
int64_t rst_debug_seq_ws_bytes(int64_t n);

/* The dispatch-rate probe: `launches` empty kernels (blocks x threads) on
 * each of nstreams fresh streams, streams interleaved; *per_s = kernels
 * completed per second (host clock, launch to the last stream's sync). */
int rst_debug_launch_rate(rst_ctx* ctx, int nstreams, int launches, int blocks, int threads,
                          double* per_s);
/* RST_TIMELINE builds (RST_DEFINES=-DRST_TIMELINE=1): the context's last
 * ICP align, per iteration and loop kernel (k_icp_nn, k_icp_fb, k_sq_tot,
 * k_sq_front, k_sq_build, k_sq_walk, k_cov_ref, k_reduce_solve) the
 * earliest wave start and the latest wave end on the 100 MHz device clock:
 * out[(iter * 8 + kernel) * 2 + {0, 1}], at most cap values; *iters = the
 * iterations run.  RST_E_STATE in other builds. */
int rst_debug_timeline(rst_ctx* ctx, uint64_t* out, int32_t cap, int32_t* iters);
/* The concurrency probe: `launches` kernels per stream on nstreams fresh
 * streams, each kernel's waves waiting spin_us on the real-time clock with
 * lds_bytes of dynamic LDS; *overlap = kernels running at once on average
 * (their busy time over the wall time). */
int rst_debug_kernel_overlap(rst_ctx* ctx, int nstreams, int launches, int blocks, int threads,
                             int spin_us, int lds_bytes, double* overlap);

/* A device stream copy (the measured HBM ceiling the rooflines are read
 * against): `bytes` copied buffer to buffer by float4 kernels (1-8 float4
 * per thread in flight, nontemporal or default policy), reps launches of
 * each variant timed with HIP events; *gbps = (read + write bytes) / the
 * best launch's time. */
int rst_debug_stream_copy(rst_ctx* ctx, int64_t bytes, int reps, double* gbps);

/* The target's leaf table: lstart[0 .. nleaves] (leaf L holds sorted
 * positions [lstart[L], lstart[L+1])) copied to the host when cap >=
 * nleaves + 1, and pleaf[0 .. m) (the leaf of each sorted position) when
 * pleaf is not NULL; *nleaves receives the leaf count either way. */
int rst_debug_target_leaves(rst_ctx* ctx, const rst_target* tgt, int32_t* lstart, int32_t cap,
                            int32_t* pleaf, int32_t* nleaves);

/* The two halves of one sharded ICP iteration (rst_icp_align_sharded_device
 * runs them with an RCCL all-reduce between), for testing the shard
 * decomposition without a second GPU.
 *
 * rst_debug_icp_partials: the partial sums of source shard `src` against
 * tgt at the given state (pose column-major 4x4, mu, the WHOLE source's
 * centroid smean, iteration index `iter`): exact NN of every shard point,
 * then the fixed-order reduction -- the vector a rank contributes to the
 * all-reduce.  *nv receives its length (16 for RST_P2POINT_REF, 30 for
 * RST_P2PLANE); out holds >= 32 doubles.  RST_P2POINT_REF needs sum_mode
 * RST_SUM_FP64 (sequential sums have no shard decomposition: RST_E_ARG).
 *
 * rst_debug_icp_solve: the solve step every rank runs on the all-reduced
 * vector (n_total = points of all shards): state in -> the next pose, mu and
 * iteration count out, exactly as the loop's k_solve_only. */
int rst_debug_icp_partials(rst_ctx* ctx, const rst_target* src, const rst_target* tgt,
                           const rst_icp_opts* opts, const float pose[16], float mu,
                           const float smean[3], int32_t iter, double* out, int32_t* nv);
int rst_debug_icp_solve(rst_ctx* ctx, const rst_icp_opts* opts, int64_t n_total,
                        const double* totals, const float smean[3], float pose_inout[16],
                        float* mu_inout, int32_t* iter_inout);

/* The rehash schedule DownsampleVoxel / ExtractPointCloud's reference order
 * is replayed from (voxel.hip umap_schedule: libstdc++'s _Prime_rehash_policy
 * for a default-constructed std::unordered_map receiving n distinct keys):
 * out[2k] = elements before the insert that rehashed, out[2k + 1] = the new
 * bucket count, at most cap pairs; *count = the number of rehashes.  Host
 * only (no GPU call). */
int rst_debug_umap_schedule(int64_t n, int64_t* out, int64_t cap, int64_t* count);

#ifdef __cplusplus
}
#endif
#endif /* RST_DEBUG_H_ */
