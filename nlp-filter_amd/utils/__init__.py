"""Mirror of kingdwd/nlp-filter ``utils`` entry points on the hot path:
``utils.ekf`` (EKF on libmhe.so) and the ``utils.gnss`` filter plug-ins."""
