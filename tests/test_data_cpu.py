"""Data pipeline vs the reference's own samplers/collate run on the same inputs
(fixture g5_data.pt, tools/gen_golden.py::gen_data): batches must be identical index lists."""

import numpy as np
import pytest
import torch

from dphubert_amd.data import (AudioDataset, BucketizeBatchSampler, CollateFnAudio, DistributedBatchSampler,
                               read_manifest)
from helpers import load_golden


@pytest.fixture(scope="module")
def fx():
    return load_golden("g5_data.pt")


def _lists(ts):
    return [t.tolist() for t in ts]


def test_token_budget_batches(fx):
    bs = BucketizeBatchSampler(fx["lengths"].tolist(), num_buckets=50, max_token_count=900000, min_len=32000,
                               max_len=250000, shuffle=False)
    assert bs.iter_list == _lists(fx["token_batches"])
    assert all(sum(fx["lengths"][i].item() for i in b) <= 900000 for b in bs.iter_list)


def test_fixed_size_batches_drop_last(fx):
    bs = BucketizeBatchSampler(fx["lengths"].tolist(), num_buckets=20, batch_size=7, min_len=32000, max_len=250000,
                               shuffle=False, drop_last=True)
    assert bs.iter_list == _lists(fx["size_batches"])


def test_shuffled_buckets_follow_global_rng(fx):
    torch.manual_seed(11)
    bs = BucketizeBatchSampler(fx["lengths"].tolist(), num_buckets=50, max_token_count=900000, min_len=32000,
                               max_len=250000, shuffle=True)
    assert bs.iter_list == _lists(fx["shuffled_token_batches"])


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("drop", [False, True])
def test_distributed_split(fx, world, drop):
    bs = BucketizeBatchSampler(fx["lengths"].tolist(), num_buckets=50, max_token_count=900000, min_len=32000,
                               max_len=250000, shuffle=False)
    seen = []
    for r in range(world):
        ds = DistributedBatchSampler(bs, num_replicas=world, rank=r, shuffle=True, seed=3, drop_last=drop)
        assert ds.subset == _lists(fx[f"dist_w{world}_d{int(drop)}_r{r}"])
        assert len(ds) == len(ds.subset)
        seen.append(len(ds))
    assert len(set(seen)) == 1          # every rank takes the same number of batches


def test_collate_crop_and_pad(fx):
    batch = [(w, w.shape[1]) for w in fx["collate_in"]]
    torch.manual_seed(13)
    w, ln = CollateFnAudio(pad=False, rand_crop=True)(batch)
    assert torch.equal(w, fx["collate_crop"][0]) and torch.equal(ln, fx["collate_crop"][1])
    w, ln = CollateFnAudio(pad=True, rand_crop=False)(batch)
    assert torch.equal(w, fx["collate_pad"][0]) and torch.equal(ln, fx["collate_pad"][1])


def test_manifest_and_wav_reader(tmp_path):
    from scipy.io import wavfile
    root = tmp_path / "audio"
    root.mkdir()
    rng = np.random.default_rng(0)
    lens = [32000, 40000]
    for i, n in enumerate(lens):
        wavfile.write(root / f"u{i}.wav", 16000, (rng.standard_normal(n) * 3000).astype(np.int16))
    (tmp_path / "train100.tsv").write_text(f"{root}\n" + "".join(f"u{i}.wav\t{n}\n" for i, n in enumerate(lens)))
    paths, got = read_manifest(tmp_path / "train100.tsv")
    assert got == lens and paths[1].endswith("u1.wav")
    ds = AudioDataset(tmp_path, "train100")
    w, n = ds[1]
    assert w.shape == (1, 40000) and n == 40000 and w.dtype == torch.float32 and w.abs().max() < 1.0
    (tmp_path / "bad.tsv").write_text(f"{root}\nx.flac\t100\n")
    with pytest.raises(NotImplementedError):
        AudioDataset(tmp_path, "bad")[0]
