"""oracle/ -- TEST INFRASTRUCTURE ONLY.

A CPU (numpy/scipy) restatement of the reference's hot path
(TobiasHoffmannP/PUC-Fluidsimulation-Project, code/StokesColor.py,
code/StokesFood.py, code/poisson.py, code/heatEq.py).  Every function cites the
reference file:line it restates.

Pinning: tests/test_oracle_golden.py checks this restatement against the golden
fixtures in tests/golden/*.npz, which were produced by running the reference
itself in the build container (tests/golden/gen_golden.py).  The one deliberate
departure is the pressure solve (SURVEY.md §0 finding 1, §8c): the reference's
pressure matrix is singular and its LU result is rounding-determined, so the
oracle solves the well-posed symmetric periodic-merged restatement instead; that
row of the parity contract is pinned only at the reference's measured noise
floor.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / the timed CPU baseline.  The product
(puc-fluidsimulation-project_amd/) never imports it.
"""
from .fem_ref import *  # noqa: F401,F403
