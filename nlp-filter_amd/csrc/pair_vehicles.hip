// Vehicle and multi-receiver pairs: kinematic bicycle (C4, nlp/dynamics.py:117-136),
// the dynamic bicycle with clock bias (autonomous-car.py, nlp/dynamics.py:148-174),
// multi_receiver (nlp/dynamics.py:81-96) and gnss_two_receiver (:98-115) with
// mixed rows (C5 / gnss-multi-receiver.py).
#include "mhe_core.h"

namespace mhe {
const PairOps* pairs_vehicles(int dyn, int meas) {
  if (dyn == MHE_DYN_KINEMATIC_BICYCLE && meas == MHE_MEAS_PSEUDORANGE)
    return pair_ops<DynKinematicBicycle, MeasPseudorange<6>>();
  // autonomous-car.py:190-213 (vehicle_dynamics_and_gnss + vehicle_pseudorange)
  if (dyn == MHE_DYN_VEHICLE_GNSS && meas == MHE_MEAS_VEHICLE_PSEUDORANGE)
    return pair_ops<DynVehicleGnss, MeasVehiclePseudorange>();
  if (meas != MHE_MEAS_MIXED) return nullptr;
  switch (dyn) {
    case MHE_DYN_KINEMATIC_BICYCLE: return pair_ops<DynKinematicBicycle, MeasMixed<6>>();
    case MHE_DYN_MULTI_RECEIVER: return pair_ops<DynMultiReceiver, MeasMixed<8>>();
    case MHE_DYN_GNSS_TWO_RECEIVER: return pair_ops<DynGnssTwoReceiver, MeasMixed<10>>();
    case MHE_DYN_VEHICLE_GNSS: return pair_ops<DynVehicleGnss, MeasMixed<9>>();
  }
  return nullptr;
}
}  // namespace mhe
