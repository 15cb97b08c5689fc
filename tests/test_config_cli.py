"""train.py's command line: every TrainConfig field parses to its declared type (Optional[int]
fields such as --max-steps-per-epoch included)."""
import argparse

from pgdist.config import TrainConfig, add_cli_args, preset


def _parse(argv):
    return add_cli_args(argparse.ArgumentParser()).parse_args(argv)


def test_optional_numeric_fields_parse_as_numbers():
    a = _parse(["--max-steps-per-epoch", "80", "--lr", "0.1", "--epochs", "3", "--watchdog-s", "5"])
    assert a.max_steps_per_epoch == 80 and isinstance(a.max_steps_per_epoch, int)
    assert a.lr == 0.1 and a.epochs == 3
    assert isinstance(a.watchdog_s, float)


def test_bool_and_str_fields():
    a = _parse(["--deterministic", "true", "--bn-sync", "broadcast", "--betas", "0.8", "0.99"])
    assert a.deterministic is True and a.bn_sync == "broadcast" and a.betas == [0.8, 0.99]


def test_unset_fields_keep_preset_defaults():
    a = _parse([])
    cfg = preset("mpi", **{k: v for k, v in vars(a).items() if v is not None})
    assert cfg == preset("mpi")
    assert isinstance(cfg, TrainConfig) and cfg.bn_sync == "broadcast"
