"""CPU oracle — TEST INFRASTRUCTURE ONLY.

This package is a plain numpy / C restatement of the reference algorithms on the
hot path (SEGNN / PONITA / EGNN-MC forwards, the self-feed rollout, the GravitySim
integrator and the fully-connected graph builder).  It exists only to CHECK the
HIP product path:

* only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
  ``bench.py`` may import it;
* nothing in the product package imports it, and the product path never falls
  back to it.

Pinning status (see DESIGN.md "Oracle"):

* graph builder, GravitySim           — pinned bit-/ulp-close against golden
  vectors produced by running the reference's own code (tests/golden/).
* PONITA, EGNN-MC forwards + rollout — pinned against golden vectors produced
  by the reference model code (with a PyG ``propagate`` test shim, see
  tests/golden/make_golden.py).
* SEGNN                                — e3nn 0.5.1 is not installable here, so
  the e3nn arithmetic is restated from its published algorithm
  (e3nn_lite.py).  Parity vs e3nn itself is UNPINNED; it is guarded by
  known-answer tests (parameter count, equivariance, closed-form paths,
  normalize2mom constants).
"""
