"""Training data feed of distill.py: manifest, token-budget batching, rank split,
crop-to-minimum collate, pinned host buffers.

Behaviour follows dataset/audio_dataset.py of the reference:
  * ``BucketizeBatchSampler``  audio_dataset.py:19-142 — keep lengths in [min_len, max_len], sort by
    length, cut ``num_buckets`` equal-width length buckets (bucket edges linspace(min_len-1,
    max_len+1)), optionally permute inside each bucket once, then pack greedily in bucket order
    until the next sample would exceed ``max_token_count`` samples (or ``batch_size`` items);
  * ``DistributedBatchSampler`` audio_dataset.py:145-217 — permute the batch list with a seeded
    generator (seed + epoch), pad by repetition (or drop the tail) to a multiple of the world
    size, rank r takes batches r, r+W, r+2W, ...;
  * ``AudioDataset``            audio_dataset.py:220-277 — ``{subset}.tsv``: first line the audio
    root, then ``relative_path<TAB>num_samples`` per line (prepare_data.py:36-50);
  * ``CollateFnAudio``          audio_dataset.py:280-363 — crop every waveform of the mini-batch to
    the shortest one (random offset when ``rand_crop``) or zero-pad to the longest.

Audio decoding: the reference uses torchaudio (absent here); 16-bit / float WAV files are read
with scipy, other containers (flac) raise — decode them to WAV offline.
"""

from pathlib import Path
from typing import Iterator, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
import torch.distributed as dist


class BucketizeBatchSampler:
    """Length-bucketed batches of sample indices (token budget or fixed batch size)."""

    def __init__(self, lengths: Sequence[int], num_buckets: int, min_len: int = 0, max_len: Optional[int] = None,
                 max_token_count: Optional[int] = None, batch_size: Optional[int] = None, shuffle: bool = True,
                 drop_last: bool = False, generator: Optional[torch.Generator] = None):
        lengths = [int(x) for x in lengths]
        if max_len is None:
            max_len = max(lengths)
        if not 0 <= min_len <= max_len:
            raise AssertionError("``min_len`` should be non-negative and smaller than ``max_len``")
        if (max_token_count is None) == (batch_size is None):
            raise AssertionError("exactly one of ``max_token_count`` and ``batch_size`` must be set")
        if max_token_count is not None and max_len > max_token_count:
            raise AssertionError("``max_token_count`` must be >= the longest kept sample")
        kept = sorted(((n, i) for i, n in enumerate(lengths) if min_len <= n <= max_len), key=lambda t: t[0])
        if not kept:
            raise AssertionError("``lengths`` cannot be empty after filtering.")
        self.lengths = [n for n, _ in kept]
        self.indices = [i for _, i in kept]
        self.max_token_count = max_token_count
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        # equal-width length buckets over the sorted positions
        edges = torch.linspace(min_len - 1, max_len + 1, num_buckets + 1)
        ids = torch.bucketize(torch.tensor(self.lengths), edges).tolist()
        buckets = {}
        for pos, b in enumerate(ids):
            buckets.setdefault(int(b), []).append(pos)
        self.buckets = {k: torch.as_tensor(v, dtype=torch.int) for k, v in sorted(buckets.items())}
        if shuffle:
            for k in self.buckets:
                perm = torch.randperm(self.buckets[k].numel(), generator=generator)
                self.buckets[k] = self.buckets[k][perm]
        self.iter_list = self._pack()

    def _pack(self) -> List[List[int]]:
        cap = self.max_token_count if self.max_token_count else self.batch_size
        out, cur, used = [], [], 0
        for pos_list in self.buckets.values():
            for pos in pos_list.tolist():
                cost = self.lengths[pos] if self.max_token_count else 1
                if used + cost <= cap:
                    cur.append(self.indices[pos])
                    used += cost
                else:
                    out.append(cur)
                    cur, used = [self.indices[pos]], cost
        if cur and (self.max_token_count or not self.drop_last):
            out.append(cur)
        return out

    def __iter__(self) -> Iterator[List[int]]:
        return iter(self.iter_list)

    def __len__(self) -> int:
        return len(self.iter_list)


class DistributedBatchSampler:
    """Split a ``BucketizeBatchSampler``'s batches over the ranks (same batches on every run)."""

    def __init__(self, batch_sampler: BucketizeBatchSampler, num_replicas: Optional[int] = None,
                 rank: Optional[int] = None, shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        if num_replicas is None:
            num_replicas = dist.get_world_size() if dist.is_initialized() else 1
        if rank is None:
            rank = dist.get_rank() if dist.is_initialized() else 0
        self.batch_sampler = batch_sampler
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.epoch = 0
        self._split()

    def _split(self):
        batches = list(self.batch_sampler.iter_list)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            batches = [batches[i] for i in torch.randperm(len(batches), generator=g).tolist()]
        W = self.num_replicas
        if self.drop_last:
            total = len(batches) - len(batches) % W
        else:
            batches = batches + batches[:W - len(batches) % W]
            total = len(batches)
        self.num_samples = total // W
        self.subset = batches[self.rank:total:W]

    def set_epoch(self, epoch: int):
        # the reference stores the epoch but keeps the split made at construction
        self.epoch = epoch

    def __iter__(self):
        return iter(self.subset)

    def __len__(self):
        return self.num_samples


def read_manifest(tsv: Union[str, Path]) -> Tuple[List[str], List[int]]:
    """prepare_data.py manifest: first line = root dir, then ``path<TAB>num_samples``."""
    paths, lens = [], []
    with open(tsv) as f:
        root = f.readline().rstrip()
        for line in f:
            if not line.strip():
                continue
            rel, n = line.rstrip("\n").split("\t")
            paths.append(f"{root}/{rel}")
            lens.append(int(n))
    return paths, lens


def load_wav(path: str) -> torch.Tensor:
    """(1, T) float32 in [-1, 1) from a WAV file (int16/int32/float)."""
    if not str(path).lower().endswith(".wav"):
        raise NotImplementedError(f"{path}: only WAV is decodable here (torchaudio/soundfile are absent); "
                                  "convert the corpus to 16 kHz WAV")
    from scipy.io import wavfile
    sr, x = wavfile.read(path)
    if x.ndim > 1:
        x = x[:, 0]
    if x.dtype == np.int16:
        x = x.astype(np.float32) / 32768.0
    elif x.dtype == np.int32:
        x = x.astype(np.float32) / 2147483648.0
    else:
        x = x.astype(np.float32)
    return torch.from_numpy(x)[None]


class AudioDataset(torch.utils.data.Dataset):
    def __init__(self, tsv_dir: Union[str, Path], subset: str):
        self.f_list, self.len_list = read_manifest(Path(tsv_dir) / f"{subset}.tsv")

    def __len__(self):
        return len(self.f_list)

    def __getitem__(self, index):
        w = load_wav(self.f_list[index])
        if w.shape[1] != self.len_list[index]:
            raise AssertionError(f"{self.f_list[index]}: {w.shape[1]} samples, manifest says {self.len_list[index]}")
        return w, w.shape[1]


class CollateFnAudio:
    """Crop to the shortest waveform of the batch (``pad=False``) or zero-pad to the longest."""

    def __init__(self, pad: bool = False, rand_crop: bool = True, generator: Optional[torch.Generator] = None):
        self.pad = pad
        self.rand_crop = rand_crop
        self.generator = generator

    def __call__(self, batch: List[Tuple[torch.Tensor, int]]) -> Tuple[torch.Tensor, torch.Tensor]:
        sizes = [w.shape[1] for w, _ in batch]
        target = max(sizes) if self.pad else min(sizes)
        waves, lens = [], []
        for w, _ in batch:
            w = w[0]
            n = target
            off = 0
            if w.numel() > n and self.rand_crop:
                off = int(torch.randint(w.numel() - n, (1,), generator=self.generator))
            elif w.numel() < n:
                n = w.numel()
            waves.append(w[off:off + n])
            lens.append(n)
        out = torch.nn.utils.rnn.pad_sequence(waves, batch_first=True)
        return out, torch.tensor(lens)


def train_loader(tsv_dir, subset: str, seconds_per_batch: float, num_workers: int = 1, seed: int = 0,
                 rank: Optional[int] = None, world: Optional[int] = None):
    """distill.py's train dataloader (lightning.py:306-325): 1000 buckets, 2-15.6 s utterances,
    token budget = seconds_per_batch * 16 kHz, batches split over ranks, pinned host memory."""
    ds = AudioDataset(tsv_dir, subset)
    bs = BucketizeBatchSampler(ds.len_list, num_buckets=1000, max_token_count=int(seconds_per_batch * 16000),
                               min_len=32000, max_len=250000, shuffle=False)
    ds_sampler = DistributedBatchSampler(bs, num_replicas=world, rank=rank, shuffle=True, seed=seed)
    return torch.utils.data.DataLoader(ds, batch_sampler=ds_sampler, collate_fn=CollateFnAudio(pad=False),
                                       num_workers=num_workers, pin_memory=torch.cuda.is_available())


def val_loader(tsv_dir, seconds_per_batch: float, num_workers: int = 1):
    """distill.py's validation dataloader (lightning.py:326-342): the ``valid`` subset, same bucketing, no rank
    split or shuffle (callers take every world-th batch)."""
    ds = AudioDataset(tsv_dir, "valid")
    bs = BucketizeBatchSampler(ds.len_list, num_buckets=1000, max_token_count=int(seconds_per_batch * 16000),
                               min_len=32000, max_len=250000, shuffle=False)
    return torch.utils.data.DataLoader(ds, batch_sampler=bs, collate_fn=CollateFnAudio(pad=False),
                                       num_workers=num_workers, pin_memory=torch.cuda.is_available())
