// The LM's residual blocks (lm_eval.inc), built for x86-64-v3 (AVX2).
#include "lm_eval.h"

#include "../include/mp_types.h"

namespace mp {
namespace {
#include "lm_eval.inc"
} // namespace

MP_LM_EVAL_ENTRY(lm_eval_range_w4)

} // namespace mp
