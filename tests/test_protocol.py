"""DataProto semantics (mirror of the reference's tests/test_protocol_on_cpu.py behaviours). CPU only."""

import pickle
import random

import numpy as np
import pytest
import torch

from verl_amd.protocol import (
    DataProto,
    DataProtoConfig,
    TensorBatch,
    fold_batch_dim,
    pad_dataproto_to_divisor,
    union_numpy_dict,
    union_tensor_dict,
    unfold_batch_dim,
    unpad_dataproto,
)


def _dp():
    return DataProto.from_dict(tensors={"obs": torch.tensor([[1, 2], [3, 4], [5, 6]])}, non_tensors={"labels": ["a", "b", "c"]},
                               meta_info={"info": "test_info"})


def test_union():
    obs = torch.randn(10, 3)
    d1 = TensorBatch({"obs": obs, "act": torch.randn(10, 2)})
    d2 = TensorBatch({"obs": obs, "rew": torch.randn(10)})
    d = union_tensor_dict(d1, d2)
    assert set(d.keys()) == {"obs", "act", "rew"}
    with pytest.raises(AssertionError):
        union_tensor_dict(d1, TensorBatch({"obs": obs + 1}))
    a = np.random.random(5)
    b = np.array([float("nan")] * 4 + ["nan"], dtype=object)
    x = {"a": a, "b": b, "c": np.tile(b, (2, 1))}
    union_numpy_dict(x, {"a": a, "b": b.copy(), "c": np.tile(b, (2, 1))})
    with pytest.raises(AssertionError):
        union_numpy_dict(x, {"a": np.random.random(5)})


def test_constructor_batch_dims():
    d = DataProto.from_dict(tensors={"obs": torch.randn(100, 10), "act": torch.randn(100, 10, 3)})
    assert d.batch.batch_size == torch.Size([100])
    with pytest.raises(AssertionError):
        DataProto.from_dict(tensors={"obs": torch.randn(100, 10), "act": torch.randn(100, 10, 3)}, num_batch_dims=2)
    with pytest.raises(AssertionError):
        DataProto.from_dict(tensors={"obs": torch.randn(5, 2), "act": torch.randn(6, 2)})


def test_make_iterator_deterministic():
    ds = DataProto.from_dict(tensors={"obs": torch.randn(100, 10)},
                             non_tensors={"labels": [random.choice(["x", "y"]) for _ in range(100)]})
    a = list(ds.make_iterator(mini_batch_size=10, epochs=2, seed=1, dataloader_kwargs={"shuffle": True}))
    b = list(ds.make_iterator(mini_batch_size=10, epochs=2, seed=1, dataloader_kwargs={"shuffle": True}))
    assert len(a) == 20
    for x, y in zip(a, b, strict=True):
        assert torch.equal(x.batch["obs"], y.batch["obs"])
        assert np.array_equal(x.non_tensor_batch["labels"], y.non_tensor_batch["labels"])


def test_reorder_chunk_concat():
    d = DataProto.from_dict(tensors={"obs": torch.tensor([1, 2, 3, 4, 5, 6])}, non_tensors={"labels": list("abcdef")},
                            meta_info={"name": "x"})
    d.reorder(torch.tensor([3, 4, 2, 0, 1, 5]))
    assert d.batch["obs"].tolist() == [4, 5, 3, 1, 2, 6]
    assert list(d.non_tensor_batch["labels"]) == list("decabf")
    with pytest.raises(AssertionError):
        d.chunk(5)
    parts = d.chunk(2)
    assert parts[0].batch["obs"].tolist() == [4, 5, 3] and parts[0].meta_info == {"name": "x"}
    back = DataProto.concat(parts)
    assert back.batch["obs"].tolist() == [4, 5, 3, 1, 2, 6]
    assert list(back.non_tensor_batch["labels"]) == list("decabf")


def test_chunk_auto_padding():
    d = DataProto.from_dict(tensors={"obs": torch.arange(7)}, non_tensors={"l": list("abcdefg")})
    DataProtoConfig.auto_padding = True
    try:
        parts = d.chunk(3)
    finally:
        DataProtoConfig.auto_padding = False
    assert [len(p) for p in parts] == [3, 3, 1]
    assert [len(p.non_tensor_batch["l"]) for p in parts] == [3, 3, 1]


def test_pop_select_rename():
    d = DataProto.from_dict(tensors={"a": torch.zeros(4), "b": torch.ones(4)}, non_tensors={"n": list("wxyz")},
                            meta_info={"m": 1, "k": 2})
    p = d.pop(batch_keys=["a"], meta_info_keys=["m"])
    assert list(p.batch.keys()) == ["a"] and p.meta_info == {"m": 1}
    assert list(d.batch.keys()) == ["b"] and d.meta_info == {"k": 2}
    s = d.select(batch_keys=["b"], non_tensor_batch_keys=[])
    assert s.non_tensor_batch == {}
    d.rename("b", "c")
    assert "c" in d.batch.keys()
    with pytest.raises(ValueError):
        d.rename(["c"], ["x", "y"])


def test_repeat_and_sample_level_repeat():
    d = _dp()
    r = d.repeat(2, interleave=True)
    assert r.batch["obs"].tolist() == [[1, 2], [1, 2], [3, 4], [3, 4], [5, 6], [5, 6]]
    assert list(r.non_tensor_batch["labels"]) == ["a", "a", "b", "b", "c", "c"]
    r = d.repeat(2, interleave=False)
    assert r.batch["obs"].tolist() == [[1, 2], [3, 4], [5, 6], [1, 2], [3, 4], [5, 6]]
    s = d.sample_level_repeat([3, 1, 2])
    assert list(s.non_tensor_batch["labels"]) == ["a", "a", "a", "b", "c", "c"]
    s = d.sample_level_repeat(torch.tensor([1, 2, 3]))
    assert s.batch["obs"].tolist() == [[1, 2], [3, 4], [3, 4], [5, 6], [5, 6], [5, 6]]


@pytest.mark.parametrize("div,pad,obs", [(2, 1, [[1, 2], [3, 4], [5, 6], [1, 2]]), (3, 0, [[1, 2], [3, 4], [5, 6]]),
                                         (7, 4, [[1, 2], [3, 4], [5, 6], [1, 2], [3, 4], [5, 6], [1, 2]])])
def test_pad_unpad(div, pad, obs):
    d = _dp()
    p, ps = pad_dataproto_to_divisor(d, div)
    assert ps == pad and p.batch["obs"].tolist() == obs and p.meta_info == {"info": "test_info"}
    u = unpad_dataproto(p, ps)
    assert torch.equal(u.batch["obs"], d.batch["obs"])
    assert list(u.non_tensor_batch["labels"]) == ["a", "b", "c"]


def test_fold_unfold():
    d = _dp().repeat(2, interleave=True)
    f = fold_batch_dim(d, new_batch_size=3)
    assert f.batch["obs"].tolist() == [[[1, 2], [1, 2]], [[3, 4], [3, 4]], [[5, 6], [5, 6]]]
    f.reorder(torch.tensor([1, 2, 0]))
    u = unfold_batch_dim(f, batch_dims=2)
    assert u.batch["obs"].tolist() == [[3, 4], [3, 4], [5, 6], [5, 6], [1, 2], [1, 2]]
    assert list(u.non_tensor_batch["labels"]) == ["b", "b", "c", "c", "a", "a"]


def test_pickle_roundtrip_and_disk(tmp_path):
    d = _dp()
    e = pickle.loads(pickle.dumps(d))
    assert torch.equal(e.batch["obs"], d.batch["obs"]) and e.meta_info == d.meta_info
    path = tmp_path / "d.pkl"
    d.save_to_disk(str(path))
    f = DataProto.load_from_disk(str(path))
    assert list(f.non_tensor_batch["labels"]) == ["a", "b", "c"]


@pytest.mark.parametrize("kind", ["np_int", "torch_int", "list_int", "np_bool", "torch_bool", "list_bool"])
def test_index_forms(kind):
    n = 20
    obs = torch.randn(n, 3)
    labels = np.array([f"l{i}" for i in range(n)], dtype=object)
    d = DataProto.from_dict(tensors={"obs": obs}, non_tensors={"labels": labels})
    rng = np.random.RandomState(0)
    idx = {
        "np_int": rng.randint(0, n, 6),
        "torch_int": torch.from_numpy(rng.randint(0, n, 6)),
        "list_int": [int(x) for x in rng.randint(0, n, 6)],
        "np_bool": rng.randint(0, 2, n).astype(bool),
        "torch_bool": torch.from_numpy(rng.randint(0, 2, n).astype(bool)),
        "list_bool": [bool(x) for x in rng.randint(0, 2, n)],
    }[kind]
    s = d[idx]
    ref_idx = np.asarray(idx.numpy() if isinstance(idx, torch.Tensor) else idx)
    assert torch.equal(s.batch["obs"], obs[torch.as_tensor(ref_idx)])
    assert np.array_equal(s.non_tensor_batch["labels"], labels[ref_idx])
    assert isinstance(s.batch.batch_size, torch.Size) and all(isinstance(v, int) for v in s.batch.batch_size)


def test_slice_int_len_and_no_batch():
    d = _dp()
    assert len(d) == 3 and len(d[1:]) == 2 and len(d[::2]) == 2
    item = d[1]
    assert item.batch["obs"].tolist() == [3, 4] and item.non_tensor_batch["labels"] == "b"
    nb = DataProto.from_dict(non_tensors={"labels": ["a", "b", "c"]}, meta_info={"info": 1})
    assert len(nb) == 3
    p = nb.pop(non_tensor_batch_keys=["labels"])
    assert list(p.non_tensor_batch["labels"]) == ["a", "b", "c"] and nb.non_tensor_batch == {}


def test_split_matches_reference_micro_batching():
    d = DataProto.from_dict(tensors={"x": torch.arange(10)})
    assert [m.batch["x"].tolist() for m in d.split(4)] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]


def test_plan_packing_pad_multiple_appends_one_dummy_sequence():
    """dp_actor._plan_packing(pad_multiple): packed length rounded up by ONE extra sequence whose
    rows are never selected; the real tokens' packing is unchanged (host logic, CPU)."""
    import numpy as np
    import torch

    from verl_amd.workers.actor.dp_actor import _plan_packing

    rs = np.random.RandomState(0)
    B, P, R = 5, 7, 9
    am = np.zeros((B, P + R), dtype=np.int64)
    for i in range(B):
        p, r = rs.randint(1, P + 1), rs.randint(1, R + 1)
        am[i, P - p : P + r] = 1
    base = _plan_packing(am, R, "cpu")
    pk = _plan_packing(am, R, "cpu", pad_multiple=16)
    nnz = int(am.sum())
    assert pk.pad == (-nnz) % 16 and (nnz + pk.pad) % 16 == 0
    assert torch.equal(pk.token_idx, base.token_idx)
    assert torch.equal(pk.sel_hidden, base.sel_hidden) and torch.equal(pk.sel_out, base.sel_out)
    assert torch.equal(pk.cu_seqlens[: B + 1], base.cu_seqlens)
    if pk.pad:
        assert len(pk.cu_seqlens) == B + 2 and int(pk.cu_seqlens[-1]) == nnz + pk.pad
        ids = torch.arange(B * (P + R)).view(B, P + R) + 1
        pos = torch.arange(P + R).repeat(B, 1)
        gi, gp = pk.gather(ids, pos)
        assert len(gi) == nnz + pk.pad and (gi[nnz:] == 0).all()
        assert torch.equal(gp[nnz:], torch.arange(pk.pad))
    assert _plan_packing(am, R, "cpu", pad_multiple=1).pad == 0


def test_plan_packing_gathers_mrope_position_ids():
    """Qwen2-VL mrope ids [B, 3, S] pack to [3, T] in the same token order as the ids
    (dp_actor.py:106-121: transpose to (3, B, S), index the (B S) tokens, (3, 1, T)); the dummy
    sequence gets 0..pad-1 on all three rows."""
    import numpy as np
    import torch

    from verl_amd.workers.actor.dp_actor import _plan_packing

    rs = np.random.RandomState(1)
    B, P, R = 4, 6, 5
    am = np.zeros((B, P + R), dtype=np.int64)
    for i in range(B):
        am[i, P - rs.randint(1, P + 1) : P + rs.randint(1, R + 1)] = 1
    pk = _plan_packing(am, R, "cpu", pad_multiple=8)
    ids = torch.arange(B * (P + R)).view(B, P + R)
    pos3 = torch.stack([ids * 10, ids * 10 + 1, ids * 10 + 2], dim=1)  # [B, 3, S], row c tagged c
    gi, gp = pk.gather(ids, pos3)
    nnz = int(am.sum())
    assert gp.shape == (3, nnz + pk.pad)
    for c in range(3):
        assert torch.equal(gp[c, :nnz], gi[:nnz] * 10 + c)
        assert torch.equal(gp[c, nnz:], torch.arange(pk.pad))
    # reference form: (3, B, S) -> rows of the flattened (B S) at the real tokens
    ref = pos3.transpose(0, 1).reshape(3, -1)[:, torch.from_numpy(np.flatnonzero(am.reshape(-1)))]
    assert torch.equal(gp[:, :nnz], ref)


def test_rewritten_helpers_keep_the_reference_error_surface():
    import numpy as np
    import pytest
    import torch

    from verl_amd.protocol import DataProto, DataProtoConfig, TensorBatch, union_numpy_dict, union_tensor_dict

    with pytest.raises(AssertionError, match="enabled must be a boolean"):
        DataProtoConfig.auto_padding = 1
    DataProtoConfig.auto_padding = True
    assert DataProtoConfig.auto_padding is True
    DataProtoConfig.auto_padding = False
    a = TensorBatch({"x": torch.zeros(2)})
    with pytest.raises(AssertionError, match="identical batch size"):
        union_tensor_dict(a, TensorBatch({"y": torch.zeros(3)}))
    with pytest.raises(AssertionError, match="x in tensor_dict1 and tensor_dict2 are not the same object"):
        union_tensor_dict(a, TensorBatch({"x": torch.ones(2)}))
    merged = union_tensor_dict(a, TensorBatch({"x": torch.zeros(2), "y": torch.ones(2)}))
    assert list(merged.keys()) == ["x", "y"]
    with pytest.raises(AssertionError, match="u in tensor_dict1"):
        union_numpy_dict({"u": np.array([1, 2], dtype=object)}, {"u": np.array([1, 3], dtype=object)})
    nan = np.array([float("nan")], dtype=object)
    assert union_numpy_dict({"v": nan}, {"v": nan.copy()})["v"] is not None
    with pytest.raises(ValueError, match="Unsupported type in data"):
        DataProto.from_single_dict({"x": torch.zeros(2), "bad": [1, 2]})
    with pytest.raises(AssertionError, match="Not all the tensor in tensors have the same batch size"):
        DataProto.from_dict(tensors={"a": torch.zeros(2), "b": torch.zeros(3)})
    d = DataProto.from_dict(tensors={"a": torch.zeros(2)}, non_tensors={"n": [1, 2]})
    assert d.non_tensor_batch["n"].dtype == object
    with pytest.raises(TypeError, match="keys must be a list or a string"):
        d.rename(old_keys=1, new_keys="b")
    with pytest.raises(ValueError, match="must have the same length"):
        d.rename(old_keys=["a"], new_keys=["b", "c"])
    with pytest.raises(AssertionError):
        d.pop(batch_keys=["missing"])
    with pytest.raises(AssertionError, match="repeat_times type must be in"):
        d.sample_level_repeat({1: 2})
    r = d.sample_level_repeat(np.array([2, 1]))
    assert len(r) == 3 and r.non_tensor_batch["n"].tolist() == [1, 1, 2]


def test_plan_packing_masked_tail_labels_follow_the_rolled_stream():
    """The last real token of a row whose response is shorter than R keeps its log-prob, labelled as
    the reference's torch.roll(input_ids_rmpad, -1) labels it (dp_actor.py:131-137): the first real
    token of the next row of the reference's micro-batch, the first row's for the last row."""
    from verl_amd.workers.actor.dp_actor import _plan_packing

    P, R = 3, 4
    S = P + R
    # rows: prompt lengths 2, 3, 1, 2; response lengths 4 (full), 2, 1, 3
    am = np.zeros((4, S), dtype=np.int64)
    for r, (pl, rl) in enumerate([(2, 4), (3, 2), (1, 1), (2, 3)]):
        am[r, P - pl : P + rl] = 1
    first = am.argmax(axis=1)
    for groups, nxt in ((None, {1: 2, 2: 3, 3: 0}), ([0, 2, 4], {1: 0, 2: 3, 3: 2})):
        pk = _plan_packing(am, R, "cpu", groups=groups)
        sel_out = pk.sel_out.numpy()
        lab = pk.label_idx.numpy()
        for o, li in zip(sel_out, lab):
            r, t = divmod(int(o), R)
            p = S - R - 1 + t
            assert am[r, p] == 1
            if am[r, p + 1]:
                assert li == r * S + p + 1
            else:  # the tail: one per short row
                assert li == nxt[r] * S + first[nxt[r]], (groups, r, t, li)
        # every real predictor position is kept, padding ones are not
        kept = {(int(o) // R, int(o) % R) for o in sel_out}
        want = {(r, t) for r in range(4) for t in range(R) if am[r, S - R - 1 + t]}
        assert kept == want


def test_unfold_column_chunks_and_future_and_env_padding(monkeypatch):
    """protocol.py:816-853 (unfold_column_chunks), :905-950 (DataProtoFuture, here over
    concurrent.futures instead of Ray object refs), :52-55 (VERL_AUTO_PADDING)."""
    from concurrent.futures import ThreadPoolExecutor

    from verl_amd.protocol import DataProto, DataProtoFuture

    d = DataProto.from_dict({"x": torch.arange(12).view(2, 6), "y": torch.tensor([10, 20])},
                            non_tensors={"z": np.array([[1, 2, 3, 4], [5, 6, 7, 8]], dtype=object),
                                         "w": np.array(["a", "b"], dtype=object)})
    u = d.unfold_column_chunks(2, split_keys=["x", "z"])
    assert len(u) == 4
    assert u.batch["x"].tolist() == [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9, 10, 11]]
    assert u.batch["y"].tolist() == [10, 10, 20, 20]
    assert u.non_tensor_batch["z"].tolist() == [[1, 2], [3, 4], [5, 6], [7, 8]]
    assert u.non_tensor_batch["w"].tolist() == ["a", "a", "b", "b"]
    r = d.unfold_column_chunks(3)  # no split keys: every key repeated
    assert r.batch["x"].shape == (6, 6) and r.non_tensor_batch["w"].tolist() == ["a"] * 3 + ["b"] * 3

    with ThreadPoolExecutor(2) as ex:
        futs = [ex.submit(lambda i=i: d.select_idxs([i])) for i in range(2)]
        fut = DataProtoFuture.concat(futs)
        whole = fut.get()
        assert whole.batch["y"].tolist() == [10, 20]
        parts = fut.chunk(2)
        assert [p.get().batch["y"].tolist() for p in parts] == [[10], [20]]

    three = DataProto.from_dict({"a": torch.arange(3)})
    with pytest.raises(AssertionError, match="only support equal chunk"):
        three.chunk(2)
    monkeypatch.setenv("VERL_AUTO_PADDING", "1")
    assert three.is_padding_enabled()
    assert [len(c) for c in three.chunk(2)] == [2, 1]


@pytest.mark.parametrize("case", ["2d", "2d_nested_labels", "3d"])
def test_unfold_column_chunks_reference_cases(case):
    """The three cases of tests/test_protocol_on_cpu.py:416-480 (inputs and expected outputs)."""
    from verl_amd.protocol import DataProto

    rows = torch.arange(1, 13).view(3, 4)
    if case == "3d":
        obs1 = torch.stack([rows, rows], dim=-1)  # [[[1, 1], [2, 2], ...], ...]
        obs2 = obs1[:, :2]
    else:
        obs1, obs2 = rows, rows[:, :2]
    labels = [["a1", "a2"], ["b1", "b2"], ["c1", "c2"]] if case == "2d_nested_labels" else ["a", "b", "c"]
    d = DataProto.from_dict(tensors={"obs1": obs1, "obs2": obs2}, non_tensors={"labels": labels},
                            meta_info={"name": "abc"})
    keys = ["obs1", "labels"] if case == "2d_nested_labels" else ["obs1"]
    u = d.unfold_column_chunks(2, split_keys=keys)
    want1 = torch.arange(1, 13).view(6, 2)
    if case == "3d":
        want1 = torch.stack([want1, want1], dim=-1)
    assert torch.equal(u.batch["obs1"], want1)
    assert torch.equal(u.batch["obs2"], torch.repeat_interleave(obs2, 2, dim=0))
    want_l = [["a1"], ["a2"], ["b1"], ["b2"], ["c1"], ["c2"]] if case == "2d_nested_labels" else list("aabbcc")
    assert (u.non_tensor_batch["labels"] == np.array(want_l, dtype=object)).all()
    assert u.meta_info == {"name": "abc"}
