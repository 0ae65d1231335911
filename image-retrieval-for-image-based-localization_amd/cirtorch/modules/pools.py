"""Reference path ``cirtorch/modules/pools.py`` (POOLING_LAYERS at :200-207).

GeM / MAC / SPoC run on the engine.  GeMmp, RMAC and ROIpool are out of scope
for this build (unused by every config, RMAC's region loop is
mis-indented upstream at ``pools.py:105-113``); they raise on construction.
"""

from ..layers.pooling import GeM, MAC, SPoC  # noqa: F401


def _out_of_scope(name):
    def make(*args, **kwargs):
        raise NotImplementedError("%s pooling is out of scope for the MI355X engine (see DESIGN.md)" % name)
    return make


GeMmp = _out_of_scope("GeMmp")
RMAC = _out_of_scope("RMAC")
Rpool = _out_of_scope("ROIpool")

POOLING_LAYERS = {
    "MAC": MAC,
    "SPoC": SPoC,
    "GeM": GeM,
    "GeMmp": GeMmp,
    "RMAC": RMAC,
    "ROIpool": Rpool,
}
