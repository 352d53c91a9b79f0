// Eight GNSS receivers (n = 40): the per-receiver block of
// gnss_two_receiver (nlp/dynamics.py:98-115) x 8, with mixed rows (pseudoranges per
// receiver, 3-D ranges between adjacent receivers).  Large-system path only.
#include "mhe_core.h"

namespace mhe {
const PairOps* pairs_receivers(int dyn, int meas) {
  if (dyn == MHE_DYN_GNSS_8_RECEIVERS && meas == MHE_MEAS_MIXED) return pair_ops<DynGnssReceivers<8>, MeasMixed<40>>();
  return nullptr;
}
}  // namespace mhe
