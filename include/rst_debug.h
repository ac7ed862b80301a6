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
 * fallback-queue length (queries no adjacency level certified), then the
 * lanes certified at level 1 without / after a walk, at level 2, level 3. */
int rst_debug_queue_trace(rst_ctx* ctx, int32_t* out, int32_t n);

#ifdef __cplusplus
}
#endif
#endif /* RST_DEBUG_H_ */
