"""Debug: NaN in the pre-norm forward (fp32 residual stream) of tests/test_ops_gpu.py::test_ffn_compaction_matches_full_width[True]."""
import copy
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")))
import torch  # noqa: E402
from dphubert_amd.synthetic import HUBERT_BASE_CONFIG  # noqa: E402
from dphubert_amd.trainer import seeded_model  # noqa: E402
DEV = "cuda"


def check(name):
    def hook(mod, inp, out):
        outs = out if isinstance(out, (tuple, list)) else (out,)
        for o in outs:
            if torch.is_tensor(o) and o.is_floating_point():
                torch.cuda.synchronize()
                print(f"   {name:60s} {tuple(o.shape)} {o.dtype} finite={bool(torch.isfinite(o).all())} "
                      f"max={float(o.float().abs().max()):.4g}", flush=True)
    return hook


for la_mode in ["init", "zeros"]:
    for compact in ["0"]:
        os.environ["DPH_FFN_COMPACT"] = compact
        cfg = copy.deepcopy(HUBERT_BASE_CONFIG)
        cfg.update(encoder_num_layers=2, encoder_projection_dropout=0.0, encoder_attention_dropout=0.0,
                   encoder_ff_interm_dropout=0.0, encoder_dropout=0.0, encoder_layer_drop=0.0,
                   encoder_prune_feed_forward_intermediate=True, encoder_layer_norm_first=True)
        torch.manual_seed(0)
        wave = (torch.randn(2, 16000 * 2) * 0.1).to(DEV)
        m = seeded_model(cfg, 0).to(DEV).train()
        g = torch.Generator().manual_seed(3)
        for name, mod in m.named_modules():
            if name.endswith("hard_concrete_for_intermediate"):
                n = mod.log_alpha.numel()
                if la_mode == "zeros":
                    la = torch.full((n,), -10.0)
                    keep = torch.randperm(n, generator=g)[:701]
                    la[keep] = torch.randn(701, generator=g) * 2.0
                    with torch.no_grad():
                        mod.log_alpha.copy_(la.to(DEV))
                mod.set_noise((torch.rand(n, generator=g) * 0.98 + 0.01).to(DEV))
        hooks = [mod.register_forward_hook(check(name)) for name, mod in m.named_modules()
                 if name.count(".") <= 4 and name]
        print(la_mode, compact, "extract_features", flush=True)
        hs, _ = m.extract_features(wave)
        print(la_mode, compact, "forward", flush=True)
        x, _ = m(wave)
        torch.cuda.synchronize()
        for h in hooks:
            h.remove()
