"""CLI flag handling: every flag a mode ignores is rejected loudly (VERDICT r2 #3 / ADVICE r2: the PS sweep
configs asked for Adam and silently ran SGD), and the r-of-50 sweep configs launch 50 gradient workers."""
import glob
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _args(argv):
    from pytorch_distributed_nn_amd.cli import parse_args
    return parse_args(argv)


@pytest.mark.parametrize("argv,mode,world", [
    (["--mode", "ps", "--graph", "on"], "ps", 3),
    (["--mode", "ps", "--straggler-mode"], "ps", 3),
    (["--mode", "ddp", "--evaluator"], "ddp", 2),
    (["--mode", "ddp", "--n-to-collect", "2"], "ddp", 2),
    (["--mode", "ddp", "--comm-type", "Async"], "ddp", 2),
    (["--mode", "single", "--save-model-secs", "5"], "single", 1),
    (["--mode", "single", "--interval-ms", "50"], "single", 1),
])
def test_ignored_flags_are_rejected(argv, mode, world):
    from pytorch_distributed_nn_amd.cli import check_mode_flags
    with pytest.raises(SystemExit) as e:
        check_mode_flags(_args(argv), mode, world)
    assert "does not use" in str(e.value)


@pytest.mark.parametrize("argv,mode,world", [
    (["--mode", "ps", "--optimizer", "adam", "--n-to-collect", "2", "--evaluator"], "ps", 4),
    (["--mode", "ddp", "--straggler-mode", "--num-aggregate", "1", "--interval-ms", "20"], "ddp", 2),
    (["--mode", "ddp", "--comm-type", "AllReduce", "--graph", "on"], "ddp", 2),
    ([], "single", 1),                      # reference defaults (num-aggregate 5, momentum 0.5) are fine
])
def test_used_flags_pass(argv, mode, world):
    from pytorch_distributed_nn_amd.cli import check_mode_flags
    check_mode_flags(_args(argv), mode, world)


def test_every_shipped_config_is_consistent():
    """Each YAML config parses and uses only flags its mode implements."""
    from pytorch_distributed_nn_amd.cli import check_mode_flags
    for cfg in glob.glob(os.path.join(ROOT, "configs", "**", "*.yaml"), recursive=True):
        a = _args(["--config", cfg])
        mode = a.mode or "single"
        world = {"ps": 4, "ddp": 2}.get(mode, 1)
        check_mode_flags(a, mode, world)


def test_sweep_configs_reproduce_r_of_50():
    """r-of-50 sweeps: 50 gradient workers + master + evaluator, Adam, evaluator on (time_loss_out_*)."""
    from sweep import nproc_for
    for cfg in glob.glob(os.path.join(ROOT, "configs", "sweeps", "*.yaml")):
        a = _args(["--config", cfg])
        assert a.optimizer == "adam" and a.evaluator and a.ps_workers == 50, cfg
        assert nproc_for(cfg, 3) == 52
        if "interval" in cfg:
            assert a.num_aggregate == 0 and a.interval_ms > 0
        else:
            assert 1 <= a.n_to_collect <= 50
