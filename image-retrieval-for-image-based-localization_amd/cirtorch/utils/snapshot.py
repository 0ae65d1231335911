"""Checkpoint I/O (reference ``cirtorch/utils/snapshot.py:6-75``).

``resume_from_snapshot(model, path, ["body", "ret_head"])`` is how the in-tree
evaluation loads weights (``scripts/train_globalF.py:797``).  Two file formats
are accepted:

* the in-tree ``save_snapshot`` dict: ``{"config", "state_dict": {module:
  state_dict, ...}, "training_meta"}`` (``snapshot.py:6-17``);
* the upstream ``{"meta", "state_dict"}`` checkpoint that ``scripts/test.py``
  loads (``:95-106``): one flat state dict of the whole network, split here by
  ``"<module>."`` key prefix.

Files are read with ``torch.load(..., weights_only=True)`` (tensors and plain
containers only; nothing in the file is executed).  Loading follows the
reference's tolerant rule (``_load_pretraining_dict``): entries whose shape
differs from the module's are dropped and missing keys are ignored.  The
engine modules rebuild their packed weights after a load.
"""

import torch

from .misc import config_to_string


def save_snapshot(file, config, epoch, last_score, best_score, global_step, **kwargs):
    data = {
        "config": config_to_string(config),
        "state_dict": dict(kwargs),
        "training_meta": {
            "epoch": epoch,
            "last_score": last_score,
            "best_score": best_score,
            "global_step": global_step,
        },
    }
    torch.save(data, file)


def _load(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def _module_state(state_dict, module):
    """the state dict of `module`: a nested entry (save_snapshot format) or the
    flat whole-network dict's "<module>." keys (upstream format); None if absent"""
    if module in state_dict and isinstance(state_dict[module], dict):
        return state_dict[module]
    prefix = module + "."
    sub = {k[len(prefix):]: v for k, v in state_dict.items() if k.startswith(prefix)}
    return sub or None


def pre_train_from_snapshots(model, snapshots, modules):
    for snapshot in snapshots:
        if ":" in snapshot:
            module_name, snapshot = snapshot.split(":")
        else:
            module_name = None
        state_dict = _load(snapshot)["state_dict"]
        if module_name is None:
            for module_name in modules:
                sd = _module_state(state_dict, module_name)
                if sd is not None:
                    _load_pretraining_dict(getattr(model, module_name), sd)
        else:
            if module_name not in modules:
                raise ValueError("Unrecognized network module {}".format(module_name))
            sd = _module_state(state_dict, module_name)
            if sd is None:  # an explicitly named module must be in the file (reference snapshot.py:35-36)
                raise KeyError("The given snapshot does not contain a state_dict for module '{}'".format(module_name))
            _load_pretraining_dict(getattr(model, module_name), sd)


def resume_from_snapshot(model, snapshot, modules):
    snapshot = _load(snapshot)
    state_dict = snapshot["state_dict"]
    for module in modules:
        sd = _module_state(state_dict, module)
        if sd is None:
            raise KeyError("The given snapshot does not contain a state_dict for module '{}'".format(module))
        _load_pretraining_dict(getattr(model, module), sd)
    return snapshot


def _load_pretraining_dict(model, state_dict):
    """``model.load_state_dict(state_dict, strict=False)`` that also drops
    entries whose shape differs from the model's (``snapshot.py:54-75``)."""
    state_dict = dict(state_dict)
    for k, v in model.state_dict().items():
        if k in state_dict and v.shape != state_dict[k].shape:
            del state_dict[k]
    model.load_state_dict(state_dict, False)
