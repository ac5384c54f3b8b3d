"""The data-parallel step through the FULL Trainer at world size 2 (two ranks on one GPU, gloo: SUM + divide, the
twin of the RCCL AVG path), each rank with its own bucketed batch length (audio_dataset.py:145-217): the reduced
gradients equal the mean of the ranks' local gradients, the bucket collectives launch in the same order on both
ranks, and the parameters stay bitwise identical across ranks after every optimizer step (distill.py:41 strategy
"ddp"); with gradient accumulation (run_large.sh's --accum_grad) and bf16 bucket payloads too.  Runs
tools/ddp_trainer_probe.py in a child process (its own process group and spawned ranks)."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("accum,comm", [(1, "fp32"), (3, "fp32"), (1, "bf16")])
def test_trainer_ws2_different_bucket_lengths(accum, comm):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, str(root / "tools" / "ddp_trainer_probe.py"), "--port", str(port),
                        "--accum", str(accum), "--comm", comm],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(root))
    out = r.stdout + r.stderr
    print(r.stdout)
    assert r.returncode == 0, out[-3000:]
    assert "DDP_TRAINER_OK" in out, out[-3000:]
