"""Subset of reference ``cirtorch/utils/misc.py`` on the extraction path:
``Empty`` (:18-20), ``try_index`` (:261-265), ``config_to_string`` (:121-125)
and ``norm_act_from_config`` (:175-235), which defines the backbone's BN +
activation for ``make_model`` (``scripts/train_globalF.py:252,257-259``)."""

import io
from functools import partial

from ..modules.abn import ABN, ActivatedAffine, InPlaceABN, InPlaceABNSync


class Empty(Exception):
    """Exception to facilitate handling of empty predictions (``utils/misc.py:18-20``)."""


def try_index(scalar_or_list, i):
    try:
        return scalar_or_list[i]
    except TypeError:
        return scalar_or_list


def config_to_string(config):
    """A ``configparser.ConfigParser`` as INI text (the ``"config"`` entry of a snapshot);
    strings pass through, None gives ""."""
    if config is None:
        return ""
    if isinstance(config, str):
        return config
    with io.StringIO() as sio:
        config.write(sio)
        return sio.getvalue()


def _get(section, key, conv, default):
    """configparser section (``getfloat`` / ``getint``) or plain mapping"""
    getter = getattr(section, {float: "getfloat", int: "getint"}[conv], None)
    if getter is not None:
        v = getter(key)
        return default if v is None else v
    v = section.get(key, default) if hasattr(section, "get") else default
    return default if v is None else conv(v)


def norm_act_from_config(body_config):
    """(norm_act_static, norm_act_dynamic) from a ``[body]`` config section with
    ``normalization_mode``, ``activation``, ``activation_slope`` and ``gn_groups``.

    Eval-mode semantics on this engine: ``bn``, ``syncbn`` and ``syncbn+bn``
    (InPlaceABN / InPlaceABNSync) and ``off`` (ActivatedAffine: the same
    inference BN + activation) all fold into the convolution epilogue, so they
    yield the same ``ABN`` partial with the configured activation and slope.
    Group normalisation (``gn``, ``syncbn+gn``) is not a per-channel affine at
    inference and is out of scope: it raises ``NotImplementedError``; an
    unknown mode raises ``ValueError`` with the reference's message."""
    mode = body_config["normalization_mode"]
    activation = body_config["activation"]
    slope = _get(body_config, "activation_slope", float, 0.01)
    if mode == "bn":
        static = dynamic = partial(InPlaceABN, activation=activation, activation_param=slope)
    elif mode == "syncbn":
        static = dynamic = partial(InPlaceABNSync, activation=activation, activation_param=slope)
    elif mode == "syncbn+bn":
        static = partial(InPlaceABNSync, activation=activation, activation_param=slope)
        dynamic = partial(InPlaceABN, activation=activation, activation_param=slope)
    elif mode == "off":
        static = dynamic = partial(ActivatedAffine, activation=activation, activation_param=slope)
    elif mode in ("gn", "syncbn+gn"):
        raise NotImplementedError("group normalisation (%r) is out of scope for the MI355X engine" % mode)
    else:
        raise ValueError("Unrecognized normalization_mode {}, valid options: 'bn', 'syncbn', 'syncbn+bn', 'gn', "
                         "'syncbn+gn', 'off'".format(mode))
    if activation not in ("leaky_relu", "relu", "identity"):
        raise NotImplementedError("activation %r is not supported by the MI355X engine" % activation)
    return static, dynamic


__all__ = ["Empty", "try_index", "config_to_string", "norm_act_from_config", "ABN"]
