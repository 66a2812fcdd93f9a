"""DataProto — the batch type that crosses every boundary of the actor-update path.

Mirror of verl/protocol.py:207-964 (DataProto, DataProtoItem, pad/unpad, union, chunk, split,
concat, repeat, reorder, select, pop, rename, padding), without tensordict or ray:
``batch`` is a :class:`TensorBatch` — an ordered dict of tensors sharing dim 0 —, and
``non_tensor_batch`` holds numpy object arrays of the same length. ``meta_info`` is a plain
dict. The pickled form is a dict of tensors written by ``torch.save`` (loaded back with
``weights_only=True``), numpy arrays and meta_info.
"""

from __future__ import annotations

import copy
import io
import logging
import pathlib
import pickle
from collections.abc import Callable, Iterator
from dataclasses import dataclass, field
from typing import Any, Optional

import numpy as np
import torch

__all__ = ["DataProto", "DataProtoItem", "TensorBatch", "union_tensor_dict", "pad_dataproto_to_divisor",
           "unpad_dataproto", "DataProtoConfig", "collate_fn", "DataProtoFuture"]



# DataProto.to(cuda) of a host batch keeps the host tensor of this key next to the device one
HOST_MIRRORED_KEY = "attention_mask"

class _TypedSwitches(type):
    """Class-level boolean switches: ``DataProtoConfig.auto_padding = True`` is type-checked on
    assignment (the reference's metaclass property, protocol.py:33-45; same message)."""

    def __setattr__(cls, name, value):
        if name in cls._switches and not isinstance(value, bool):
            raise AssertionError(f"enabled must be a boolean, got {value} as {type(value)}")
        super().__setattr__(name, value)


class DataProtoConfig(metaclass=_TypedSwitches):
    """Global switch for auto-padding in chunk() (protocol.py:47-63); a batch can also opt in
    through ``meta_info[auto_padding_key]``."""

    _switches = ("auto_padding",)
    auto_padding = False
    auto_padding_key = "_verl_auto_padding"


class TensorBatch(dict):
    """Ordered mapping of tensors with a common leading batch dimension (TensorDict stand-in)."""

    def __init__(self, source: Optional[dict] = None, batch_size=None):
        super().__init__()
        source = source or {}
        for k, v in source.items():
            if not isinstance(v, torch.Tensor):
                raise TypeError(f"TensorBatch values must be tensors, got {type(v)} for {k}")
            dict.__setitem__(self, k, v)
        if batch_size is None:
            batch_size = (next(iter(source.values())).shape[0],) if source else (0,)
        if isinstance(batch_size, int):
            batch_size = (batch_size,)
        self.batch_size = torch.Size(batch_size)
        for k, v in self.items():
            if tuple(v.shape[: len(self.batch_size)]) != tuple(self.batch_size):
                raise ValueError(f"key {k} has shape {tuple(v.shape)}, batch size is {tuple(self.batch_size)}")

    def __setitem__(self, key, value):
        if not isinstance(value, torch.Tensor):
            raise TypeError("TensorBatch values must be tensors")
        if tuple(value.shape[: len(self.batch_size)]) != tuple(self.batch_size):
            raise ValueError(f"key {key}: shape {tuple(value.shape)} does not match batch size {tuple(self.batch_size)}")
        dict.__setitem__(self, key, value)

    def __getitem__(self, item):
        if isinstance(item, str):
            return dict.__getitem__(self, item)
        sel = {k: v[item] for k, v in self.items()}
        n = next(iter(sel.values())).shape[0] if sel else _index_len(item, self.batch_size[0])
        return TensorBatch(sel, batch_size=(n,))

    @property
    def device(self):
        devs = {v.device for v in self.values()}
        return devs.pop() if len(devs) == 1 else None

    def to(self, device) -> "TensorBatch":
        return TensorBatch({k: v.to(device) for k, v in self.items()}, batch_size=self.batch_size)

    def select(self, *keys) -> "TensorBatch":
        return TensorBatch({k: dict.__getitem__(self, k) for k in keys}, batch_size=self.batch_size)

    def pop(self, key, *default):
        return dict.pop(self, key, *default)

    def rename_key_(self, old_keys, new_keys):
        for o, n in zip(old_keys, new_keys, strict=True):
            dict.__setitem__(self, n, dict.pop(self, o))
        return self

    def contiguous(self) -> "TensorBatch":
        return TensorBatch({k: v.contiguous() for k, v in self.items()}, batch_size=self.batch_size)

    def chunk(self, chunks: int, dim: int = 0) -> list["TensorBatch"]:
        assert dim == 0
        parts = {k: torch.chunk(v, chunks, dim=0) for k, v in self.items()}
        n = len(next(iter(parts.values()))) if parts else 0
        return [TensorBatch({k: p[i] for k, p in parts.items()}) for i in range(n)]

    def update_from(self, tensors: dict) -> "TensorBatch":
        """Insert several tensors (batch size checked per key), keeping insertion order."""
        for k, v in tensors.items():
            self[k] = v
        return self

    def clone(self) -> "TensorBatch":
        return TensorBatch({k: v.clone() for k, v in self.items()}, batch_size=self.batch_size)

    @property
    def sorted_keys(self):
        return sorted(self.keys())

    def __repr__(self):
        body = ", ".join(f"{k}: {tuple(v.shape)} {v.dtype}" for k, v in self.items())
        return f"TensorBatch(batch_size={tuple(self.batch_size)}, {{{body}}})"


def _key_list(keys):
    """None, one key or a list of keys -> None or a list (rename's argument forms)."""
    if keys is None or isinstance(keys, list):
        return keys
    if isinstance(keys, str):
        return [keys]
    raise TypeError(f"keys must be a list or a string, but got {type(keys)}")


def _index_len(item, n):
    if isinstance(item, slice):
        return len(range(*item.indices(n)))
    return len(item)


def _cat_batches(batches: list[TensorBatch]) -> TensorBatch:
    keys = list(batches[0].keys())
    return TensorBatch({k: torch.cat([b[k] for b in batches], dim=0) for k in keys})


def union_tensor_dict(tensor_dict1: TensorBatch, tensor_dict2: TensorBatch) -> TensorBatch:
    """protocol.py:105-118: add ``tensor_dict2``'s keys to ``tensor_dict1`` in place; a key held by
    both must hold equal tensors (AssertionError texts as the reference)."""
    if tensor_dict1.batch_size != tensor_dict2.batch_size:
        raise AssertionError(f"Two tensor dict must have identical batch size. Got {tensor_dict1.batch_size} "
                             f"and {tensor_dict2.batch_size}")
    shared = [k for k in tensor_dict2 if k in tensor_dict1]
    differing = next((k for k in shared if not tensor_dict1[k].equal(tensor_dict2[k])), None)
    if differing is not None:
        raise AssertionError(f"{differing} in tensor_dict1 and tensor_dict2 are not the same object")
    tensor_dict1.update_from({k: v for k, v in tensor_dict2.items() if k not in tensor_dict1})
    return tensor_dict1


def _arrays_equal(a: np.ndarray, b: np.ndarray) -> bool:
    if a.shape != b.shape:
        return False
    for x, y in zip(a.reshape(-1), b.reshape(-1), strict=True):
        both_nan = isinstance(x, float) and isinstance(y, float) and np.isnan(x) and np.isnan(y)
        if not both_nan and not np.array_equal(np.asarray(x, dtype=object), np.asarray(y, dtype=object)):
            return False
    return True


def union_numpy_dict(d1: dict, d2: dict) -> dict:
    """protocol.py:121-132: merge object arrays into ``d1``; shared keys must hold equal arrays
    (NaN == NaN for this purpose)."""
    for key in d1.keys() & d2.keys():
        a, b = d1[key], d2[key]
        if not (isinstance(a, np.ndarray) and isinstance(b, np.ndarray)) or not _arrays_equal(b, a):
            raise AssertionError(f"{key} in tensor_dict1 and tensor_dict2 are not the same object")
    d1.update(d2)
    return d1


def union_two_dict(dict1: dict, dict2: dict) -> dict:
    """meta_info merge: shared keys must be equal."""
    clash = next((k for k in dict2 if k in dict1 and dict1[k] != dict2[k]), None)
    if clash is not None:
        raise AssertionError(f"{clash} in meta_dict1 and meta_dict2 are not the same object")
    dict1.update(dict2)
    return dict1


def list_of_dict_to_dict_of_list(list_of_dict: list[dict]) -> dict:
    """[{k: v_i}] -> {k: [v_i]}; every dict must carry only the first dict's keys."""
    keys = list(list_of_dict[0]) if list_of_dict else []
    if any(set(d) - set(keys) for d in list_of_dict):
        raise AssertionError("list_of_dict entries carry keys the first entry does not have")
    return {k: [d[k] for d in list_of_dict if k in d] for k in keys}


@dataclass
class DataProtoItem:
    batch: Optional[TensorBatch] = None
    non_tensor_batch: dict = field(default_factory=dict)
    meta_info: dict = field(default_factory=dict)


def collate_fn(x: list[DataProtoItem]) -> "DataProto":
    batch = TensorBatch({k: torch.stack([it.batch[k] for it in x]) for k in x[0].batch.keys()})
    non_tensor = {k: np.array([it.non_tensor_batch[k] for it in x], dtype=object) for k in x[0].non_tensor_batch}
    return DataProto(batch=batch, non_tensor_batch=non_tensor, meta_info=x[0].meta_info)


@dataclass
class DataProto:
    """Batch protocol (protocol.py:207). ``batch``: TensorBatch; ``non_tensor_batch``: dict of
    numpy object arrays; ``meta_info``: dict."""

    batch: Optional[TensorBatch] = None
    non_tensor_batch: dict = field(default_factory=dict)
    meta_info: dict = field(default_factory=dict)

    def __post_init__(self):
        if self.batch is not None and not isinstance(self.batch, TensorBatch):
            self.batch = TensorBatch(dict(self.batch))
        self.check_consistency()

    # ------------------------------------------------------------------ basics
    def __len__(self):
        if self.batch is not None:
            return self.batch.batch_size[0]
        if self.non_tensor_batch:
            return next(iter(self.non_tensor_batch.values())).shape[0]
        return 0

    def __getitem__(self, item):
        if isinstance(item, slice):
            return self.slice(item.start, item.stop, item.step)
        if isinstance(item, list | np.ndarray | torch.Tensor):
            return self.select_idxs(item)
        if isinstance(item, int | np.integer):
            tensor_data = TensorBatch({k: v[item] for k, v in self.batch.items()}, batch_size=()) if self.batch is not None else None
            non_tensor = {k: v[item] for k, v in self.non_tensor_batch.items()}
            return DataProtoItem(batch=tensor_data, non_tensor_batch=non_tensor, meta_info=self.meta_info)
        raise TypeError(f"Indexing with {type(item)} is not supported")

    def __getstate__(self):
        buf = io.BytesIO()
        tensors = None if self.batch is None else {k: v.contiguous() for k, v in self.batch.items()}
        torch.save(tensors, buf)
        return buf.getvalue(), self.non_tensor_batch, self.meta_info

    def __setstate__(self, data):
        raw, non_tensor_batch, meta_info = data
        tensors = torch.load(io.BytesIO(raw), weights_only=True, map_location="cpu")
        self.batch = None if tensors is None else TensorBatch(tensors)
        self.non_tensor_batch = non_tensor_batch
        self.meta_info = meta_info

    def save_to_disk(self, filepath):
        """Writes __getstate__'s form (tensors via torch.save, numpy arrays, meta_info)."""
        pathlib.Path(filepath).write_bytes(pickle.dumps(self))

    @staticmethod
    def load_from_disk(filepath) -> "DataProto":
        """Reads a file written by save_to_disk of THIS package (it unpickles: trusted files only)."""
        return pickle.loads(pathlib.Path(filepath).read_bytes())

    def print_size(self, prefix=""):
        t = sum(v.element_size() * v.numel() for v in self.batch.values()) if self.batch is not None else 0
        a = sum(v.nbytes for v in self.non_tensor_batch.values())
        msg = f"Size of tensordict: {t / 1024**3} GB, size of non_tensor_batch: {a / 1024**3} GB"
        print(f"{prefix}, {msg}" if prefix else msg)

    def check_consistency(self):
        if self.batch is not None:
            assert len(self.batch.batch_size) == 1, "only support num_batch_dims=1"
        if self.non_tensor_batch is not None:
            for key, val in self.non_tensor_batch.items():
                assert isinstance(val, np.ndarray), (
                    f"data in the non_tensor_batch must be a numpy.array with dtype=object, but for {key=}, got {type(val)=}"
                )
        if self.batch is not None and self.non_tensor_batch:
            bs = self.batch.batch_size[0]
            for key, val in self.non_tensor_batch.items():
                assert val.shape[0] == bs, f"key {key} length {len(val)} is not equal to batch size {bs}"

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_single_dict(cls, data: dict, meta_info=None, auto_padding=False):
        """Tensors go to ``batch``, numpy arrays to ``non_tensor_batch`` (protocol.py:255-268)."""
        odd = next((v for v in data.values() if not isinstance(v, torch.Tensor | np.ndarray)), None)
        if odd is not None:
            raise ValueError(f"Unsupported type in data {type(odd)}")
        return cls.from_dict(tensors={k: v for k, v in data.items() if isinstance(v, torch.Tensor)},
                             non_tensors={k: v for k, v in data.items() if isinstance(v, np.ndarray)},
                             meta_info=meta_info, auto_padding=auto_padding)

    @classmethod
    def from_dict(cls, tensors=None, non_tensors=None, meta_info=None, num_batch_dims=1, auto_padding=False):
        assert num_batch_dims > 0, "num_batch_dims must be greater than zero"
        if non_tensors is not None:
            assert num_batch_dims == 1, "only support num_batch_dims=1 when non_tensors is not None."
        tensors = tensors or {}
        meta_info = meta_info if meta_info is not None else {}
        non_tensors = non_tensors if non_tensors is not None else {}
        assert isinstance(non_tensors, dict)
        lead = {k: t.shape[:num_batch_dims] for k, t in tensors.items()}
        pivot = next(iter(lead), None)
        odd = next((k for k, sz in lead.items() if sz != lead[pivot]), None)
        if odd is not None:
            raise AssertionError(f"Not all the tensor in tensors have the same batch size with batch_dims="
                                 f"{num_batch_dims}. Got {pivot} has {lead[pivot]}, {odd} has {lead[odd]}")
        non_tensors.update({k: np.array(v, dtype=object) for k, v in non_tensors.items()
                            if not isinstance(v, np.ndarray)})
        batch = TensorBatch(tensors, batch_size=lead[pivot]) if tensors else None
        if auto_padding:
            meta_info[DataProtoConfig.auto_padding_key] = True
        return cls(batch=batch, non_tensor_batch=non_tensors, meta_info=meta_info)

    # ------------------------------------------------------------------ moves and views
    def to(self, device, non_blocking: bool = False) -> "DataProto":
        if self.batch is not None:
            moved = {}
            for k, v in self.batch.items():
                t = v.to(device, non_blocking=non_blocking)
                if k == HOST_MIRRORED_KEY and t is not v and v.device.type == "cpu" and t.is_cuda:
                    # a private host copy of the mask as it was moved: the actor plans padding removal
                    # from it instead of a device->host copy that would drain the stream
                    # (dp_actor._mask_host). A clone, not the caller's tensor: writes to that through
                    # numpy views or a reused loader buffer do not bump its version
                    t._va_host_mirror = (v.clone(), t._version)
                moved[k] = t
            self.batch = TensorBatch(moved, batch_size=self.batch.batch_size)
        return self

    def select(self, batch_keys=None, non_tensor_batch_keys=None, meta_info_keys=None, deepcopy=False) -> "DataProto":
        sub_batch = self.batch.select(*tuple(batch_keys)) if batch_keys is not None else self.batch
        if non_tensor_batch_keys is not None:
            non_tensor = {k: v for k, v in self.non_tensor_batch.items() if k in non_tensor_batch_keys}
        else:
            non_tensor = self.non_tensor_batch
        if deepcopy:
            non_tensor = copy.deepcopy(non_tensor)
        if meta_info_keys is not None:
            meta = {k: v for k, v in self.meta_info.items() if k in meta_info_keys}
        else:
            meta = self.meta_info
        if deepcopy:
            meta = copy.deepcopy(meta)
        return type(self)(batch=sub_batch, non_tensor_batch=non_tensor, meta_info=meta)

    def select_idxs(self, idxs) -> "DataProto":
        if isinstance(idxs, list):
            idxs = torch.tensor(idxs)
            if idxs.dtype != torch.bool:
                idxs = idxs.type(torch.int32)
        if isinstance(idxs, np.ndarray):
            idxs_np, idxs_t = idxs, torch.from_numpy(idxs)
        else:
            idxs_t, idxs_np = idxs, idxs.detach().cpu().numpy()
        n = int(idxs_np.sum()) if idxs_np.dtype == bool else idxs_np.shape[0]
        batch = None
        if self.batch is not None:
            dev = self.batch.device
            it = idxs_t.to(dev) if dev is not None else idxs_t
            batch = TensorBatch({k: v[it] for k, v in self.batch.items()}, batch_size=(n,))
        non_tensor = {k: v[idxs_np] for k, v in self.non_tensor_batch.items()}
        return type(self)(batch=batch, non_tensor_batch=non_tensor, meta_info=self.meta_info)

    def slice(self, start=None, end=None, step=None) -> "DataProto":
        s = slice(start, end, step)
        batch = self.batch[s] if self.batch is not None else None
        non_tensor = {k: v[s] for k, v in self.non_tensor_batch.items()}
        return type(self)(batch=batch, non_tensor_batch=non_tensor, meta_info=self.meta_info)

    def pop(self, batch_keys=None, non_tensor_batch_keys=None, meta_info_keys=None) -> "DataProto":
        """Remove the named keys from this batch and return them as a new DataProto."""
        def take(store, keys):
            missing = [k for k in keys or [] if k not in store]
            if missing:
                raise AssertionError(f"keys {missing} not present")
            return {k: store.pop(k) for k in keys or []}

        return DataProto.from_dict(tensors=take(self.batch, batch_keys),
                                   non_tensors=take(self.non_tensor_batch, non_tensor_batch_keys),
                                   meta_info=take(self.meta_info, meta_info_keys))

    def rename(self, old_keys=None, new_keys=None) -> "DataProto":
        """Rename batch keys in place (protocol.py:420-445; same TypeError / ValueError texts)."""
        old_keys, new_keys = _key_list(old_keys), _key_list(new_keys)
        if len(new_keys) != len(old_keys):
            raise ValueError(
                f"new_keys and old_keys must have the same length, but got {len(new_keys)} and {len(old_keys)}")
        self.batch.rename_key_(tuple(old_keys), tuple(new_keys))
        return self

    def union(self, other: "DataProto") -> "DataProto":
        if self.batch is None:
            self.batch = other.batch
        elif other.batch is not None:
            self.batch = union_tensor_dict(self.batch, other.batch)
        self.non_tensor_batch = union_numpy_dict(self.non_tensor_batch, other.non_tensor_batch)
        self.meta_info = union_two_dict(self.meta_info, other.meta_info)
        return self

    def make_iterator(self, mini_batch_size, epochs, seed=None, dataloader_kwargs=None) -> Iterator["DataProto"]:
        """protocol.py:625-663 — mini-batch iterator; shuffles when dataloader_kwargs['shuffle']."""
        assert len(self) % mini_batch_size == 0, f"{len(self)} % {mini_batch_size} != 0"
        kw = dataloader_kwargs or {}
        gen = torch.Generator()
        if seed is not None:
            gen.manual_seed(seed)

        def gen_data():
            for _ in range(epochs):
                order = torch.randperm(len(self), generator=gen) if kw.get("shuffle", False) else torch.arange(len(self))
                for s in range(0, len(self), mini_batch_size):
                    d = self.select_idxs(order[s : s + mini_batch_size])
                    d.meta_info = self.meta_info
                    yield d

        return iter(gen_data())

    # ------------------------------------------------------------------ padding / chunking
    def is_padding_enabled(self) -> bool:
        """protocol.py:52-55 / 681-687: the batch's meta_info flag, the class switch, or the
        VERL_AUTO_PADDING environment variable (TRUE / 1)."""
        import os

        env = os.getenv("VERL_AUTO_PADDING", "FALSE").upper() in ("TRUE", "1")
        return bool(self.meta_info.get(DataProtoConfig.auto_padding_key, False) or DataProtoConfig.auto_padding or env)

    def padding(self, padding_size, padding_candidate=""):
        if padding_size == 0:
            return
        cand = self.select_idxs([0 if padding_candidate == "first" else len(self) - 1])
        padded = DataProto.concat([self, cand.repeat(padding_size)])
        self.batch = padded.batch
        self.non_tensor_batch = padded.non_tensor_batch

    def chunk(self, chunks: int) -> list["DataProto"]:
        """protocol.py:689-728 — equal chunks along dim 0 (DP_COMPUTE_PROTO dispatch)."""
        if not self.is_padding_enabled():
            assert len(self) % chunks == 0, f"only support equal chunk. Got size of DataProto {len(self)} and chunk {chunks}."
        if self.batch is not None:
            batch_lst = self.batch.chunk(chunks=chunks, dim=0)
            sizes = np.array([b.batch_size[0] for b in batch_lst])
            cuts = np.cumsum(sizes)[:-1]
        else:
            batch_lst = [None] * chunks
            sizes, cuts = None, None
        non_tensor_lst = [{} for _ in range(chunks)]
        for key, val in self.non_tensor_batch.items():
            parts = np.array_split(val, cuts.tolist()) if sizes is not None else np.array_split(val, chunks)
            assert len(parts) == chunks
            for i in range(chunks):
                non_tensor_lst[i][key] = parts[i]
        return [type(self)(batch=batch_lst[i], non_tensor_batch=non_tensor_lst[i], meta_info=self.meta_info)
                for i in range(chunks)]

    def split(self, split_size: int) -> list["DataProto"]:
        return [self[i : i + split_size] for i in range(0, len(self), split_size)]

    @staticmethod
    def concat(data: list["DataProto"]) -> "DataProto":
        new_batch = _cat_batches([d.batch for d in data]) if data[0].batch is not None else None
        non_tensor = list_of_dict_to_dict_of_list([d.non_tensor_batch for d in data])
        for key, val in non_tensor.items():
            non_tensor[key] = np.concatenate(val, axis=0)
        cls = type(data[0]) if data else DataProto
        return cls(batch=new_batch, non_tensor_batch=non_tensor, meta_info=data[0].meta_info)

    def reorder(self, indices):
        idx_np = indices.detach().cpu().numpy()
        self.batch = self.batch[indices.to(self.batch.device) if self.batch.device is not None else indices]
        self.non_tensor_batch = {k: v[idx_np] for k, v in self.non_tensor_batch.items()}

    def repeat(self, repeat_times=2, interleave=True) -> "DataProto":
        """protocol.py:772-814 — interleave=True keeps each prompt's n samples contiguous."""
        batch = None
        if self.batch is not None:
            if interleave:
                rep = {k: v.repeat_interleave(repeat_times, dim=0) for k, v in self.batch.items()}
            else:
                rep = {k: v.unsqueeze(0).expand(repeat_times, *v.shape).reshape(-1, *v.shape[1:])
                       for k, v in self.batch.items()}
            batch = TensorBatch(rep, batch_size=(self.batch.batch_size[0] * repeat_times,))
        non_tensor = {}
        for key, val in self.non_tensor_batch.items():
            non_tensor[key] = np.repeat(val, repeat_times, axis=0) if interleave else np.tile(
                val, (repeat_times,) + (1,) * (val.ndim - 1))
        return type(self)(batch=batch, non_tensor_batch=non_tensor, meta_info=self.meta_info)

    def unfold_column_chunks(self, n_split: int, split_keys: Optional[list] = None) -> "DataProto":
        """protocol.py:816-853: the keys in ``split_keys`` are split along dim 1 into n_split parts
        unfolded into the batch dim ([B, n k, ...] -> [B n, k, ...], row-major); every other key
        (tensor and non-tensor) is repeated n_split times per row (repeat_interleave)."""
        keys = set(split_keys) if split_keys is not None else set()

        def unfold(x):
            shape = list(x.shape)
            shape[0], shape[1] = x.shape[0] * n_split, x.shape[1] // n_split
            return x.reshape(*shape)

        batch = None
        if self.batch is not None:
            src = {k: (unfold(v) if k in keys else torch.repeat_interleave(v, n_split, dim=0))
                   for k, v in self.batch.items()}
            batch = TensorBatch(src, batch_size=(len(self) * n_split,))
        non_tensor = {k: (unfold(v) if k in keys else np.repeat(v, n_split, axis=0))
                      for k, v in self.non_tensor_batch.items()}
        return type(self)(batch=batch, non_tensor_batch=non_tensor, meta_info=self.meta_info)

    def sample_level_repeat(self, repeat_times) -> "DataProto":
        """protocol.py:855-901 — per-sample repeat counts (list / tuple / 1-D tensor or array)."""
        if isinstance(repeat_times, torch.Tensor | np.ndarray):
            if repeat_times.ndim != 1:
                raise AssertionError(f"repeat_times must be 1-D, got {repeat_times.ndim} dims")
            repeat_times = repeat_times.tolist()
        elif not isinstance(repeat_times, list | tuple):
            raise AssertionError(
                f"repeat_times type must be in [list, torch.Tensor, np.ndarray, tuple], got {type(repeat_times)}")
        repeat_times = [int(r) for r in repeat_times]
        reps = torch.tensor(repeat_times)
        batch = None
        if self.batch is not None:
            rep = {k: v.repeat_interleave(reps.to(v.device), dim=0) for k, v in self.batch.items()}
            batch = TensorBatch(rep, batch_size=(int(reps.sum()),))
        non_tensor = {k: np.repeat(v, repeat_times, axis=0) for k, v in self.non_tensor_batch.items()}
        return type(self)(batch=batch, non_tensor_batch=non_tensor, meta_info=self.meta_info)


def pad_dataproto_to_divisor(data: DataProto, size_divisor: int):
    """protocol.py:70-95 — pad by re-using leading rows; returns (padded, pad_size)."""
    assert isinstance(data, DataProto), "data must be a DataProto"
    if len(data) % size_divisor != 0:
        pad_size = size_divisor - len(data) % size_divisor
        parts, remaining = [], pad_size
        while remaining > 0:
            take = min(remaining, len(data))
            parts.append(data[:take])
            remaining -= take
        return DataProto.concat([data] + parts), pad_size
    if len(data) == 0:
        logging.warning("padding a DataProto with no item, no changed made")
    return data, 0


def unpad_dataproto(data: DataProto, pad_size):
    return data[:-pad_size] if pad_size != 0 else data


def fold_batch_dim(data: DataProto, new_batch_size):
    """protocol.py:147-164."""
    bs = data.batch.batch_size[0]
    assert bs % new_batch_size == 0
    tensors = {k: v.view(new_batch_size, -1, *v.shape[1:]) for k, v in data.batch.items()}
    non_tensor = {k: np.reshape(v, (new_batch_size, -1, *v.shape[1:])) for k, v in data.non_tensor_batch.items()}
    out = DataProto(batch=None, non_tensor_batch={}, meta_info=data.meta_info)
    out.batch = TensorBatch(tensors, batch_size=(new_batch_size,))
    out.non_tensor_batch = non_tensor
    return out


def unfold_batch_dim(data: DataProto, batch_dims=2):
    """protocol.py:167-183 — inverse of fold_batch_dim: merge the leading ``batch_dims`` dims."""
    tensors = {k: v.reshape(-1, *v.shape[batch_dims:]) for k, v in data.batch.items()}
    non_tensor = {k: np.reshape(v, (-1, *v.shape[batch_dims:])) for k, v in data.non_tensor_batch.items()}
    out = DataProto(batch=None, non_tensor_batch={}, meta_info=data.meta_info)
    out.batch = TensorBatch(tensors) if tensors else None
    out.non_tensor_batch = non_tensor
    return out


@dataclass
class DataProtoFuture:
    """protocol.py:905-950 without Ray: a list of per-worker results to be collected (collect_fn,
    DataProto.concat by default) and optionally re-partitioned (dispatch_fn) on get(). A future is
    anything with .result() (concurrent.futures) or an already computed DataProto; this process runs
    no Ray object store, so ray.get becomes .result()."""

    collect_fn: Callable
    futures: list
    dispatch_fn: Optional[Callable] = None

    @staticmethod
    def concat(data: list) -> "DataProtoFuture":
        return DataProtoFuture(collect_fn=DataProto.concat, futures=data)

    def chunk(self, chunks: int) -> list["DataProtoFuture"]:
        from functools import partial

        def dispatch_fn(x, i, chunks):
            return x.chunk(chunks=chunks)[i]

        return [DataProtoFuture(collect_fn=self.collect_fn, futures=self.futures,
                                dispatch_fn=partial(dispatch_fn, i=i, chunks=chunks)) for i in range(chunks)]

    def get(self):
        output = [f.result() if hasattr(f, "result") else f for f in self.futures]
        for o in output:
            assert isinstance(o, DataProto)
        output = self.collect_fn(output)
        if self.dispatch_fn is not None:
            output = self.dispatch_fn(output)
        return output


def all_gather_data_proto(data: DataProto, process_group) -> None:
    """protocol.py:953-964 — in-place all-gather of every batch key and non-tensor array."""
    import torch.distributed as dist

    world = dist.get_world_size(group=process_group)
    if data.batch is not None:
        gathered = {}
        for k in sorted(data.batch.keys()):
            v = data.batch[k].contiguous()
            out = [torch.empty_like(v) for _ in range(world)]
            dist.all_gather(out, v, group=process_group)
            gathered[k] = torch.cat(out, dim=0)
        data.batch = TensorBatch(gathered)
    objs: list[Any] = [None] * world
    dist.all_gather_object(objs, data.non_tensor_batch, group=process_group)
    data.non_tensor_batch = {k: np.concatenate([o[k] for o in objs]) for k in data.non_tensor_batch}
