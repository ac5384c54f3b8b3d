"""CLI plumbing on CPU: the reference's launch environment (run.sh:2-9,48: srun, one task per GPU), the predlayer
heads of distill.py:100-107, and the flags (distill.py:147-331)."""

import argparse

import pytest
import torch

from dphubert_amd import cli


def test_slurm_tasks_become_torch_distributed_ranks():
    env = {"SLURM_NTASKS": "4", "SLURM_PROCID": "2", "SLURM_LOCALID": "2", "SLURM_NNODES": "1", "SLURM_JOB_ID": "777",
           "SLURM_JOB_NODELIST": "gpu07"}
    out = cli._slurm_env(env)
    assert out == {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2", "MASTER_ADDR": "127.0.0.1",
                   "MASTER_PORT": str(20000 + 777 % 20000)}
    # multi-node: the first host of the step's node list is the rendezvous
    env.update(SLURM_NTASKS="8", SLURM_PROCID="5", SLURM_LOCALID="1", SLURM_NNODES="2",
               SLURM_STEP_NODELIST="gpu[07-08]")
    out = cli._slurm_env(env)
    assert (out["WORLD_SIZE"], out["RANK"], out["LOCAL_RANK"], out["MASTER_ADDR"]) == ("8", "5", "1", "gpu07")
    # an explicit rendezvous wins; torch.distributed.run's own variables win over SLURM's
    env.update(MASTER_ADDR="10.0.0.3", MASTER_PORT="29999")
    out = cli._slurm_env(env)
    assert "MASTER_ADDR" not in out and "MASTER_PORT" not in out
    assert cli._slurm_env(dict(env, WORLD_SIZE="8")) is None
    # one task (sbatch without srun, or srun -n1): not a distributed launch
    assert cli._slurm_env({"SLURM_NTASKS": "1", "SLURM_PROCID": "0"}) is None


@pytest.mark.parametrize("nodes,first", [("n1,n2", "n1"), ("gpu[03-06,09]", "gpu03"), ("a[1-2],b7", "a1"),
                                         ("node12", "node12")])
def test_slurm_first_host(nodes, first):
    assert cli._slurm_first_host(nodes) == first


def test_no_relaunch_under_srun(monkeypatch):
    """Each srun task is one rank already: _maybe_relaunch must not start torch.distributed.run (4 tasks x 4
    workers on one port) but export the rank variables instead."""
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("SLURM_NTASKS", "4")
    monkeypatch.setenv("SLURM_PROCID", "3")
    monkeypatch.setenv("SLURM_LOCALID", "3")
    monkeypatch.setenv("SLURM_JOB_ID", "5")

    def boom(*a, **k):
        raise AssertionError("relaunched under srun")

    monkeypatch.setattr(cli.subprocess, "call", boom)
    args = argparse.Namespace(gpus=4, num_nodes=1)
    cli._maybe_relaunch(args, [])
    import os
    assert (os.environ["WORLD_SIZE"], os.environ["RANK"], os.environ["LOCAL_RANK"]) == ("4", "3", "3")


def test_predlayer_heads_and_layer2layer_sharing():
    groups, layers = cli._split_groups("0.4,8,12")
    assert layers == [0, 4, 8, 12]
    p = cli._projections(groups, 768, 768, identity=True)     # distill.py:24-26 identity init (square only)
    assert len(p) == 4 and p[1] is p[2] is p[3] and p[0] is not p[1]
    assert torch.equal(p[0].weight, torch.eye(768)) and torch.equal(p[0].bias, torch.zeros(768))
    h = cli._projections(groups, 768, 768, identity=False, mode="predlayer")
    assert len(h) == 4 and len({id(m) for m in h}) == 4
    for m in h:
        assert isinstance(m, torch.nn.Sequential) and isinstance(m[0], torch.nn.Linear) and \
            isinstance(m[1], torch.nn.GELU)
    # the reference's state_dict keys of the heads (distill_linear_projs.{i}.0.weight)
    assert "0.0.weight" in h.state_dict() and "3.0.bias" in h.state_dict()
    with pytest.raises(ValueError):
        cli._projections(groups, 768, 768, identity=False, mode="bogus")


def test_flags():
    a = cli.distill_parser().parse_args(["--distill_mode", "predlayer", "--graphs", "on", "--accum_grad", "3"])
    assert (a.distill_mode, a.graphs, a.accum_grad, a.reshuffle_each_epoch) == ("predlayer", "on", 3, False)
    a = cli.final_distill_parser().parse_args([])
    assert a.graphs == "auto" and a.distill_mode == "layer2layer"
