"""End-to-end CLI pipeline on the GPU, run.sh's four stages (run.sh:20-60): distill.py -> prune.py ->
final_distill.py -> save_final_ckpt.py, each as its own process with the reference's flags, on a 2-layer
HuBERT-Base-width model and a 16 kHz WAV manifest in prepare_data.py's tsv format (scipy-written files)."""
import copy
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _run(args):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable] + [str(a) for a in args], cwd=str(ROOT), capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, (args, r.stdout[-2000:], r.stderr[-4000:])
    return r


@pytest.mark.timeout(900)
def test_distill_prune_final_distill_save(tmp_path):
    from scipy.io import wavfile
    from dphubert_amd.cli import load_pruned_model
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG
    from dphubert_amd.trainer import seeded_model
    cfg = copy.deepcopy(HUBERT_BASE_CONFIG)
    cfg.update(encoder_num_layers=2, encoder_use_attention=[True] * 2, encoder_use_feed_forward=[True] * 2,
               encoder_num_heads=[12] * 2, encoder_ff_interm_features=[3072] * 2)
    teacher = tmp_path / "teacher.pth"
    torch.save({"config": cfg, "state_dict": seeded_model(cfg, 0).state_dict()}, teacher)
    wav_dir = tmp_path / "wav"
    wav_dir.mkdir()
    rng = np.random.default_rng(0)
    lines = [str(wav_dir)]
    for i in range(12):
        n = int(rng.integers(32000, 64000))            # 2-4 s (the loader keeps 2-15.6 s)
        wavfile.write(wav_dir / f"u{i}.wav", 16000, (rng.standard_normal(n) * 3000).astype(np.int16))
        lines.append(f"u{i}.wav\t{n}")
    (tmp_path / "train100.tsv").write_text("\n".join(lines) + "\n")
    common = ["--tsv_dir", tmp_path, "--gpus", "1", "--warmup_updates", "1", "--seconds_per_batch", "16",
              "--distill_layers", "0.1,2", "--num_workers", "0", "--log_interval", "1"]
    exp = tmp_path / "exp"
    _run(["distill.py", *common, "--teacher_ckpt", teacher, "--student_ckpt", teacher, "--exp_dir", exp,
          "--max_updates", "3", "--sparsity_warmup_updates", "2", "--target_sparsity", "0.5"])
    ck = exp / "ckpts" / "last.ckpt"
    assert ck.exists()
    state = torch.load(ck, map_location="cpu", weights_only=True)
    assert state["global_step"] == 3
    # the reference's log keys (lightning.py:277-295) plus the roofline keys of SURVEY 2 "Metrics / logging"
    recs = [json.loads(x) for x in (exp / "log.jsonl").read_text().splitlines() if x.strip()]
    train = [r for r in recs if "train_loss" in r]
    assert train and all(0.0 < r["mfma_util"] < 1.0 and r["hbm_gbps"] > 0.0 and "audio_s_per_s" in r
                         for r in train), train
    _run(["prune.py", "--distilled_ckpt", ck, "--original_ckpt", teacher])
    pruned = exp / "ckpts" / "pruned_hubert_base.pth"
    pk = torch.load(pruned, map_location="cpu", weights_only=True)
    exp2 = tmp_path / "exp2"
    _run(["final_distill.py", *common, "--teacher_ckpt", teacher, "--student_ckpt", pruned, "--exp_dir", exp2,
          "--max_updates", "2"])
    ck2 = exp2 / "ckpts" / "last.ckpt"
    assert ck2.exists()
    _run(["save_final_ckpt.py", "--config_path", pruned, "--ckpt_after_final_distill", ck2])
    final = exp2 / "ckpts" / "pruned_hubert_base.pth"
    fk = torch.load(final, map_location="cpu", weights_only=True)
    assert fk["config"] == pk["config"]
    assert set(fk["state_dict"]) == set(pk["state_dict"])
    # the final student runs on the HIP path and its weights moved during final distillation
    model = load_pruned_model(final).cuda().eval()
    w = torch.randn(2, 32000, device="cuda") * 0.1
    with torch.no_grad():
        hs, _ = model.extract_features(w)
    assert all(torch.isfinite(h.float()).all() for h in hs)
    moved = [k for k in pk["state_dict"] if pk["state_dict"][k].dtype.is_floating_point and
             not torch.equal(pk["state_dict"][k], fk["state_dict"][k])]
    assert moved, "final distillation did not update the pruned student"
