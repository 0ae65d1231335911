"""Reference path ``cirtorch/modules/normalizations.py`` (NORMALIZATION_LAYERS :30-33)."""

from ..layers.normalization import L2N  # noqa: F401


def PowerLaw(*args, **kwargs):
    raise NotImplementedError("PowerLaw normalisation is out of scope (unused by every config)")


NORMALIZATION_LAYERS = {
    "L2N": L2N,
    "PowerLaw": PowerLaw,
}
