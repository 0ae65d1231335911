"""globalFeatureAlgo (reference ``cirtorch/algos/GF_algo.py:37-94``):
selects the ``mod5`` level (or the first FPN level for list inputs) and runs
the head.  Training (``training`` / ``globalFeatureLoss``) is out of scope."""

from ..utils.misc import Empty
from ..utils.parallel import PackedSequence


class globalFeatureLoss:
    def __init__(self, name=None, sigma=0.1, epsilon=1e-6):
        self.name, self.sigma, self.epsilon = name, sigma, epsilon

    def __call__(self, *args, **kwargs):
        raise NotImplementedError("training losses are out of scope for the MI355X extract-and-match engine")


class globalFeatureAlgo:
    def __init__(self, loss, min_level, fpn_levels):
        self.loss = loss
        self.min_level = min_level
        self.fpn_levels = fpn_levels

    def _get_level(self, x):
        if isinstance(x, list):
            x = x[self.min_level:self.min_level + self.fpn_levels][0]
        elif isinstance(x, dict):
            x = x["mod5"]
        else:
            raise NameError("unknown input type")
        return x

    def _head(self, head, x):
        return head(x)

    def training(self, head, x, labels, img_size):
        raise NotImplementedError("training is out of scope for the MI355X extract-and-match engine")

    def inference(self, head, x, img_size):
        x = self._get_level(x)
        try:
            ret_pred = self._head(head, x)
        except Empty:
            ret_pred = PackedSequence([None for _ in range(x[0].size(0))])
        return ret_pred
