// gnss_pos_and_bias pairs (nlp/dynamics.py:68-79): pseudorange (C3), full_state,
// mixed rows.
#include "mhe_core.h"

namespace mhe {
const PairOps* pairs_gnss(int dyn, int meas) {
  if (dyn != MHE_DYN_GNSS_POS_AND_BIAS) return nullptr;
  switch (meas) {
    case MHE_MEAS_PSEUDORANGE: return pair_ops<DynGnssPosAndBias, MeasPseudorange<5>>();
    case MHE_MEAS_FULL_STATE: return pair_ops<DynGnssPosAndBias, MeasFullState<5>>();
    case MHE_MEAS_MIXED: return pair_ops<DynGnssPosAndBias, MeasMixed<5>>();
  }
  return nullptr;
}
}  // namespace mhe
