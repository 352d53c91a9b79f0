// Integrator pairs (nlp/dynamics.py:4-38) with full_state measurements (C1).
#include "mhe_core.h"

namespace mhe {
const PairOps* pairs_integrators(int dyn, int meas) {
  if (meas != MHE_MEAS_FULL_STATE) return nullptr;
  switch (dyn) {
    case MHE_DYN_SINGLE_INTEGRATOR: return pair_ops<DynSingleIntegrator, MeasFullState<1>>();
    case MHE_DYN_SINGLE_INTEGRATOR_2D: return pair_ops<DynSingleIntegratorND<2>, MeasFullState<2>>();
    case MHE_DYN_DOUBLE_INTEGRATOR: return pair_ops<DynDoubleIntegrator, MeasFullState<4>>();
  }
  return nullptr;
}
}  // namespace mhe
