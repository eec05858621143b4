"""TEST INFRASTRUCTURE — CPU oracle for the DPEngine.aggregate hot path.

Nothing in this package is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it, and only as the checker (or the timed CPU baseline), never as the
thing measured or shipped.  The product path (``pipelinedp_amd``) never
imports it and fails loudly when its HIP library is missing.

Modules
  columnar            vectorised NumPy restatement of bounding + per-partition
                      reduction + selection/noise, sharing the GPU's counter-based
                      priority and Philox streams (bit-exact checker).
  pydp_restatement    restatement of the python-dp (PyDP ~=1.1.5rc4) arithmetic the
                      reference calls: Gaussian sigma calibration, Laplace diversity,
                      partition-selection strategies.
  local_backend_port  row-wise restatement of LocalBackend + DPEngine.aggregate
                      (dict group-bys, np.random.choice, np.clip per pair): the CPU
                      baseline ("port") timed by bench.py.
  gen_golden          regenerates tests/golden/*.json by running the reference
                      itself in the build container (never on the GPU box).

Pinning: the oracle is checked against the reference's own known answers
(tests/test_oracle_known_answers.py) and against golden vectors produced by
the reference in this container (tests/golden/, tests/test_oracle_golden.py).
"""
