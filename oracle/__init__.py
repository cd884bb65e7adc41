"""CPU oracle for the GC-SLAM bin-path per-scan backend -- TEST INFRASTRUCTURE ONLY.

This package is a numpy float64 restatement of the reference operators on the
hot path named in BASELINE.json (the README's 14-step bin pipeline, see
SURVEY.md section 3.3 / 8).  Every function cites the reference file:line it
follows.  It exists for exactly two purposes:

  * the parity checker used by ``tests/`` and ``__graft_entry__.smoke()``;
  * the ``cpu_baseline`` leg of ``bench.py`` (kind = "port").

The product path (``gc-slam_amd/``) never imports, links or executes anything
in here; it fails loudly when its HIP library is missing.

Parity pinning: the reference is JAX (``requirements.txt:3``, jax 0.9.0) and
JAX is not installed in this image (ordinary ImportError, not a permission
denial), so the reference cannot be executed here and holds no golden vectors
for this path.  The oracle is pinned only by the
reference's own property tests (restated in ``tests/test_oracle_properties.py``)
and by closed-form known answers.  Bit-level parity with the JAX reference is
therefore **parity unpinned**; see DESIGN.md section "Oracle".
"""

from . import se3, primitives, ops, pipeline  # noqa: F401
