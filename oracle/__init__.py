"""CPU oracle for the collocation Gauss-Newton hot path -- TEST INFRASTRUCTURE ONLY.

This package is a plain NumPy restatement of the reference algorithm
(kingdwd/nlp-filter, ``nlp/collocation.py``, ``nlp/nlp.py:189-317``,
``nlp/dynamics.py``, ``nlp/measurements.py``, ``utils/ekf.py``, ``utils/gnss.py``)
used as the *checker* for the HIP path.

Rules (enforced by review, see DESIGN.md "Oracle"):
  * only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
    ``bench.py`` may import anything from here;
  * nothing in ``nlp-filter_amd/`` (the product) imports it -- the product path
    fails loudly when ``libmhe.so`` is missing instead of falling back to CPU.

Pinning: the constants (tau, D, w, poly1d phi) and the plug-in values/Jacobians
are pinned against golden vectors produced by the reference itself
(``tests/golden/gen_golden.py``, run in the build container where
``/root/reference`` exists); the EKF against the reference EKF run on the
gnss_stationary log (``tests/golden/ekf_gnss_stationary.npz``, 51 steps, bit-exact)
and against the reference EKF with autonomous-car.py's own plug-ins on 300 seeded steps
(``tests/golden/ekf_autocar.npz``, 3e-14);
the least-squares initialiser against reference runs on seeded logs and against the
stored ``data/gnss-multi-receiver/LS_{A,B}.csv`` (tests/test_multi_receiver.py).  The
stored result pickles (``ekf.pkl``, ``nlp-{l2,huber}.pkl``, ``nlp.pkl``) are NOT used:
the only loader permitted for files shipped in the reference, torch.load(weights_only=
True), refuses these Python-2 pickles.  The Gauss-Newton optimum of the
IPOPT path is NOT pinnable here (CasADi/IPOPT absent): it is checked against
``scipy.optimize.least_squares`` on the same objective instead ("parity unpinned" for
IPOPT itself); the one stored IPOPT output that can be read
(``NLP_{A,B}.csv``) is shown not to be the optimum of the script's objective.
"""
