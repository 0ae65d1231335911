"""Subset of reference ``cirtorch/utils/misc.py`` used on the hot path."""


class Empty(Exception):
    """Exception to facilitate handling of empty predictions (``utils/misc.py:18-20``)."""


def try_index(scalar_or_list, i):
    try:
        return scalar_or_list[i]
    except TypeError:
        return scalar_or_list
