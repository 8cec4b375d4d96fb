// Entry points declared in gnnrec.h whose kernels land later in this round.
#include "common.h"

extern "C" int gnnrec_score_topk_f32(const float*, int64_t, int64_t, const float*, int64_t, int64_t,
                                     int32_t, const int64_t*, const int32_t*, int32_t, int64_t*,
                                     float*, gnnrec_stream_t) {
  gnnrec::set_error("score_topk: not built yet");
  return GNNREC_EUNSUPPORTED;
}
