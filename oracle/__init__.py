"""CPU oracle for the extract-and-match hot path — TEST INFRASTRUCTURE ONLY.

This package is a plain CPU restatement (torch-CPU + numpy) of the reference
``cirtorch`` algorithm for the hot path named in BASELINE.json:

    extract: normalize -> ResNet body (mod1..mod5) -> GeM -> L2N -> Linear whiten -> L2N
    match:   scores = db . q  ->  ranks = argsort(-scores)

Every function cites the reference file:line it restates (paths relative to the
upstream repository Tarekbouamer/Image-Retrieval-for-Image-Based-Localization).

Who may use it: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — and there only as the *checker* or the
timed CPU baseline.  The product (``cirtorch`` under the package directory and
``librr.so``) never imports, links or calls anything here; on a machine without
the HIP library the product raises instead of falling back to this code.

Pinning: the restatement is checked against golden vectors produced by running
the reference modules themselves in the survey/build container
(``tests/golden/make_golden.py``; fixtures in ``tests/golden/*.npz``), see
DESIGN.md §Oracle.
"""

from . import data, ops, weights, backbone  # noqa: F401
