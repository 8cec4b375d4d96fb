// Entry points declared in gnnrec.h whose kernels land later in this round.
#include "common.h"

extern "C" int gnnrec_gat_aggregate_f32(const int64_t*, const int32_t*, int64_t, const float*,
                                        int64_t, const float*, const float*, int32_t, int32_t,
                                        float, int32_t, float*, int64_t, gnnrec_stream_t) {
  gnnrec::set_error("gat_aggregate: not built yet");
  return GNNREC_EUNSUPPORTED;
}

extern "C" int gnnrec_score_topk_f32(const float*, int64_t, int64_t, const float*, int64_t, int64_t,
                                     int32_t, const int64_t*, const int32_t*, int32_t, int64_t*,
                                     float*, gnnrec_stream_t) {
  gnnrec::set_error("score_topk: not built yet");
  return GNNREC_EUNSUPPORTED;
}
