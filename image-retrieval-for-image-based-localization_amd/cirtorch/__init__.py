"""cirtorch — MI355X-native extract-and-match engine behind the reference's
`cirtorch` operator surface (Tarekbouamer/Image-Retrieval-for-Image-Based-Localization).

Same module paths, class names and argument meanings as the reference
(cirtorch.modules.pools, cirtorch.modules.normalizations,
cirtorch.modules.heads.global_head, cirtorch.backbones, cirtorch.algos.GF_algo,
cirtorch.models.GF_net, cirtorch.utils.*) plus the upstream names that
scripts/test.py imports (cirtorch.layers.*, init_network, extract_vectors,
datahelpers, testdataset, utils.evaluate).  Compute runs in librr.so (HIP,
gfx950) through the C ABI in include/rr.h; there is no CPU fallback.
"""

__version__ = "0.1.0"
