"""Reference ``cirtorch/modules/utils.py:42-79``: output dimensionality per
architecture (``make_model`` reads ``OUTPUT_DIM[arch]`` when the FPN is off,
``scripts/train_globalF.py:331``).  The reference defines the table twice; the
second definition (``:61-79``) is the live one and is reproduced here.  Only
the ResNet rows have an engine body; the rest are kept so lookups behave the
same."""

OUTPUT_DIM = {
    "alexnet": 256,
    "vgg11": 512,
    "vgg13": 512,
    "vgg16": 512,
    "vgg19": 512,
    "resnet18": 512,
    "resnet34": 512,
    "resnet50": 2048,
    "resnet101": 2048,
    "resnet152": 2048,
    "densenet121": 1024,
    "densenet161": 2208,
    "densenet169": 1664,
    "densenet201": 1920,
    "densenet264": 2688,
    "squeezenet1_0": 512,
    "squeezenet1_1": 512,
}
