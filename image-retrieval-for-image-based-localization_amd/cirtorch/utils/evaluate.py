"""Upstream ``cirtorch.utils.evaluate`` names used by ``scripts/test.py:17,249,259``
(3-argument, printing ``compute_map_and_print``)."""

from .evaluation.ParisOxfordEval import compute_ap, compute_map  # noqa: F401
from .evaluation.ParisOxfordEval import compute_map_and_print as _cmp


def compute_map_and_print(dataset, ranks, gnd, kappas=[1, 5, 10]):
    return _cmp(dataset, ranks, gnd, kappas=kappas)
