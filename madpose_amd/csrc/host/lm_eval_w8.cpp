// The LM's residual blocks (lm_eval.inc), built for x86-64-v4 (AVX-512).
#include "lm_eval.h"

#include "../include/mp_types.h"

namespace mp {
namespace {
#include "lm_eval.inc"
} // namespace

MP_LM_EVAL_ENTRY(lm_eval_range_w8)

} // namespace mp
