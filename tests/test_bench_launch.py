"""bench.py's own rank launch: ``python bench.py --gpus N`` with no launcher starts
N torchrun ranks as a child process and returns its exit code; under a launcher, a --gpus /
WORLD_SIZE mismatch is an error.  CPU only: the child launcher is replaced by a recorder."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


@pytest.fixture
def bench(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    import bench as b
    return b


def test_gpus2_spawns_torchrun_child_with_exact_argv(bench, monkeypatch):
    seen = []

    def fake_call(argv):
        seen.append(argv)
        return 7

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(bench, "_free_port", lambda: 29577)
    args = ["--gpus", "2", "--steps", "5", "--warmup", "2"]
    monkeypatch.setattr(sys, "argv", [os.path.join(REPO, "bench.py")] + args)
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 7  # the child's exit code propagates
    assert seen == [[sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                     "--master-addr", "127.0.0.1", "--master-port", "29577",
                     os.path.join(REPO, "bench.py")] + args]


def test_child_success_exits_zero(bench, monkeypatch):
    monkeypatch.setattr(subprocess, "call", lambda argv: 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 0


def test_launcher_world_mismatch_is_an_error(bench, monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    called = []
    monkeypatch.setattr(subprocess, "call", lambda argv: called.append(argv) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 2 and not called  # no relaunch under a launcher, no 1-GPU run


def test_world_from_env_matches(bench, monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert bench.world_from_env(4) == (3, 4, 3)
    monkeypatch.delenv("WORLD_SIZE")
    monkeypatch.delenv("RANK")
    monkeypatch.delenv("LOCAL_RANK")
    assert bench.world_from_env(1) == (0, 1, 0)  # the driver's N = 1 command: unchanged


def test_real_child_launch_propagates_rc(bench, tmp_path):
    """The real subprocess path end to end, with a stand-in script instead of torchrun's ranks:
    launch_ranks runs its argv as a child and returns the child's code."""
    script = tmp_path / "child.py"
    script.write_text("import sys; print('child', sys.argv[1:]); sys.exit(3)\n")
    rc = bench.launch_ranks(2, ["--x"], run=lambda argv: subprocess.call([sys.executable, str(script)] + argv[-1:]))
    assert rc == 3
