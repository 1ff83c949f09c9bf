"""The reference package's observation helper (footsies_gym/utils.py:7-41), for single and batched
observations.

``get_dict_obs_from_vector_obs`` turns an observation that went through the observation
wrappers back into FootsiesEnv's dict form: un-flattened against the dict space it was
flattened from (gymnasium's ``FlattenObservation`` layout), then ``FootsiesNormalized.undo``.
Like the reference, it does not apply to frame-skipped observations.

The flattened layout is gymnasium's (``gymnasium.spaces.utils.flatten``): the Dict's entries in
its key order, a ``MultiDiscrete`` entry as one one-hot block per element (``nvec[i]`` wide), a
``Box`` entry raveled.  With gymnasium importable its own ``unflatten`` is used for single
observations; otherwise (and for batches: rows of a vector env's flattened observations) the
same layout is decoded here.
"""
import numpy as np

from . import spaces as _sp
from .wrappers import FootsiesNormalized


def _is_multidiscrete(space):
    return hasattr(space, "nvec")


def flat_size(space):
    """Length of gymnasium's flattened form of a Dict of MultiDiscrete / Box entries."""
    n = 0
    for sub in space.values() if hasattr(space, "values") else space.spaces.values():
        n += int(np.sum(sub.nvec)) if _is_multidiscrete(sub) else int(np.prod(sub.shape))
    return n


def _entries(space):
    return list(space.spaces.items()) if hasattr(space, "spaces") else list(space.items())


def flatten_obs(space, obs):
    """gymnasium's flatten of a dict observation (single, or batched with a leading axis)."""
    parts = []
    batched = None
    for key, sub in _entries(space):
        x = np.asarray(obs[key])
        if batched is None:
            batched = x.ndim > len(sub.shape)
        lead = x.shape[:1] if batched else ()
        if _is_multidiscrete(sub):
            nvec = np.asarray(sub.nvec).reshape(-1)
            x = x.reshape(lead + (nvec.size,)).astype(np.int64)
            for i, n in enumerate(nvec):
                parts.append(np.eye(int(n), dtype=np.float64)[x[..., i]])
        else:
            parts.append(x.reshape(lead + (-1,)).astype(np.float64))
    return np.concatenate(parts, axis=-1)


def unflatten_obs(space, flat):
    """The inverse of ``flatten_obs``: a dict with each entry in its space's shape and dtype (with
    a leading batch axis when ``flat`` is 2-D)."""
    flat = np.asarray(flat)
    if flat.shape[-1] != flat_size(space):
        raise ValueError("a flattened observation of %d values does not match the space (%d)"
                         % (flat.shape[-1], flat_size(space)))
    lead = flat.shape[:-1]
    out, at = {}, 0
    for key, sub in _entries(space):
        if _is_multidiscrete(sub):
            nvec = np.asarray(sub.nvec).reshape(-1)
            vals = []
            for n in nvec:
                vals.append(np.argmax(flat[..., at:at + int(n)], axis=-1))
                at += int(n)
            out[key] = np.stack(vals, axis=-1).reshape(lead + tuple(sub.shape)).astype(sub.dtype)
        else:
            m = int(np.prod(sub.shape))
            out[key] = flat[..., at:at + m].reshape(lead + tuple(sub.shape)).astype(sub.dtype)
            at += m
    return out


def get_dict_obs_from_vector_obs(vector_obs, flattened=True, unflattenend_observation_space=None,
                                 normalized=True, normalized_guard=True):
    """footsies_gym.utils.get_dict_obs_from_vector_obs (utils.py:7-41), with the same arguments
    (the reference's spelling of ``unflattenend_observation_space`` included) and errors:
    ValueError when ``flattened`` is set without the space, or when an unflattened observation is
    not a dict.  Also takes a batch (a 2-D array of flattened rows, or a dict of batched arrays)."""
    if flattened:
        if unflattenend_observation_space is None:
            raise ValueError("if argument vector_obs is flattened, then the unflattened observation space needs "
                             "to be provided")
        flat = np.asarray(vector_obs)
        if flat.ndim == 1 and _sp._gs is not None:  # pragma: no cover - gymnasium is absent in this image
            from gymnasium.spaces.utils import unflatten
            dict_obs = unflatten(unflattenend_observation_space, flat)
        else:
            dict_obs = unflatten_obs(unflattenend_observation_space, flat)
    elif isinstance(vector_obs, dict):
        dict_obs = vector_obs
    else:
        raise ValueError("if argument vector_obs is not flattened, it's assumed to be a dictionary (actual type: %s)"
                         % type(vector_obs).__name__)
    if normalized:
        dict_obs = FootsiesNormalized.undo(dict_obs, normalized_guard=normalized_guard)
    return dict_obs
