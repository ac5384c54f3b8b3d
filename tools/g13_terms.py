"""Where g13's loss offset comes from: the reference's own bf16 floor at 24 pre-norm Large layers (build container).

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/g13_terms.py

Re-runs the g13 step (tools/gen_golden.py gen_large24: 24 pre-norm layers, D 1024, normalize_waveform, distill layers
0.4,8,12,16,20,24, 1 x 2 s) twice by importing the reference -- exact fp32, and under Bf16Emulation (every
nn.Linear / nn.Conv1d operand and output, the LayerNorm rows, the attention P and dS rounded to bf16: what a bf16-MFMA
path does, tools/gen_golden.py:150) -- and stores the SIGNED per-term logged values of both runs plus the per-layer
hidden checksums of the emulated run in tests/golden/g13_terms.pt (data only).  tests/test_parity_gpu.py
test_g13_offset_is_the_bf16_floor compares the GPU step's signed per-term offsets with the emulation's.
"""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tools"))
sys.dont_write_bytecode = True

import gen_golden as G  # noqa: E402  (imports the reference with its stubs)


class OneSideEmulation(G.Bf16Emulation):
    """Bf16Emulation on one model only: ``side`` = "student" runs the (frozen) teacher's extract_features with the
    emulation paused, "teacher" the student's -- the noise of s - t from one side alone, uncorrelated with the
    other's (the GPU's teacher and student run different kernels: tile shapes, persistence, stream)."""

    def __init__(self, side):
        self.side = side

    def __enter__(self):
        super().__enter__()
        emu = (torch.nn.Linear.forward, torch.nn.Conv1d.forward, torch.nn.functional.softmax,
               torch.nn.functional.layer_norm)
        orig = self.orig
        cls = type(G.wav2vec2_model(**G.small_cfg(1)))
        self.cls, self.ef = cls, cls.extract_features
        ef, side = self.ef, self.side

        def wrapped(model, *a, **k):
            teacher = not any(p.requires_grad for p in model.parameters())
            pause = (teacher and side == "student") or (not teacher and side == "teacher")
            if not pause:
                return ef(model, *a, **k)
            (torch.nn.Linear.forward, torch.nn.Conv1d.forward, torch.nn.functional.softmax,
             torch.nn.functional.layer_norm) = orig
            try:
                return ef(model, *a, **k)
            finally:
                (torch.nn.Linear.forward, torch.nn.Conv1d.forward, torch.nn.functional.softmax,
                 torch.nn.functional.layer_norm) = emu

        cls.extract_features = wrapped
        return self

    def __exit__(self, *exc):
        self.cls.extract_features = self.ef
        super().__exit__(*exc)


def main():
    torch.set_num_threads(8)
    cfg = G.large_cfg(24)
    kw = dict(B=1, S=32000, units="conv,head,interm", lambdas=(0.2, 0.1), global_step=5000, sens=False)
    exact = G.run_step(cfg, cfg, "0.4,8,12,16,20,24", **kw)
    with G.Bf16Emulation():
        emu = G.run_step(cfg, cfg, "0.4,8,12,16,20,24", **kw)
    fx = torch.load(REPO / "tests" / "golden" / "g13_large24.pt", weights_only=True)
    assert abs(exact["loss"].item() - fx["loss"].item()) < 1e-6, (exact["loss"].item(), fx["loss"].item())
    out = {"loss_exact": exact["loss"].detach(), "loss_emulated": emu["loss"].detach(),
           "logged_exact": exact["logged"], "logged_emulated": emu["logged"],
           "student_hidden_ck_emulated": emu["student_hidden_ck"]}
    for side in ("student", "teacher"):
        with OneSideEmulation(side):
            one = G.run_step(cfg, cfg, "0.4,8,12,16,20,24", **kw)
        out[f"loss_emulated_{side}_only"] = one["loss"].detach()
        out[f"logged_emulated_{side}_only"] = one["logged"]
    torch.save(out, REPO / "tests" / "golden" / "g13_terms.pt")
    for side in ("student", "teacher"):
        d = {k: float(out[f"logged_emulated_{side}_only"][k]) - float(exact["logged"][k])
             for k in ("train_loss", "train_loss_l1", "train_loss_cos")}
        print(f"{side}-only emulation: " + "  ".join(f"{k} {v:+.3e}" for k, v in d.items()))
    for k in exact["logged"]:
        a, b = float(exact["logged"][k]), float(emu["logged"][k])
        print(f"{k:22s} exact {a:+.6f}  bf16-emulated {b:+.6f}  delta {b - a:+.3e}")


if __name__ == "__main__":
    main()
