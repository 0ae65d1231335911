"""Upstream ``cirtorch.utils.general`` names ``scripts/test.py:18`` imports
(reference ``cirtorch/utils/general.py:1-27``): the data root and a
human-readable duration."""

import os


def get_root():
    return os.environ.get("CIRTORCH_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__)))))


def get_data_root():
    return os.environ.get("CIRTORCH_DATA", os.path.join(get_root(), "data"))


def htime(c):
    """seconds -> "Dd Hh Mm Ss", starting at the largest non-zero unit ("5s", "2m 0s", ...)."""
    minutes, secs = divmod(round(c), 60)
    hours, mins = divmod(minutes, 60)
    days, hrs = divmod(hours, 24)
    fields = [(days, "d"), (hrs, "h"), (mins, "m"), (secs, "s")]
    first = next((i for i, (v, _) in enumerate(fields[:-1]) if v > 0), len(fields) - 1)
    return " ".join("%d%s" % f for f in fields[first:])
