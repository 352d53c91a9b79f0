// van der Pol pairs (nlp/dynamics.py:61-66): the C2 headline kernel (full_state)
// and mixed rows (large-system path).  One translation unit per pair group so
// the library builds in parallel (make -j).
#include "mhe_core.h"

namespace mhe {
const PairOps* pairs_vdp(int dyn, int meas) {
  if (dyn == MHE_DYN_VAN_DER_POL && meas == MHE_MEAS_FULL_STATE) return pair_ops<DynVanDerPol, MeasFullState<2>>();
#ifndef MHE_FAST_BUILD  // -DMHE_FAST_BUILD: the C2 kernel only (kernel development)
  if (dyn == MHE_DYN_VAN_DER_POL && meas == MHE_MEAS_MIXED) return pair_ops<DynVanDerPol, MeasMixed<2>>();
#endif
  return nullptr;
}
}  // namespace mhe
