"""CPU checks of bench.py's --gpus N launcher (the driver runs `python bench.py --gpus N` without
a launcher and with one): the parent spawns one fresh process per rank with the torchrun env
(reference src/jobs/train.sh:48 `torchrun --nproc_per_node`), forwards rank 0's JSON line, stops
the other ranks when one fails, and a WORLD_SIZE that disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402  (imports torch only: the package is imported inside main())

RANK_SCRIPT = """
import json, os, sys, time
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["MASTER_PORT"]) > 0
assert os.environ["LOCAL_RANK"] == str(r)
mode = sys.argv[1]
if mode == "fail" and r == 1:
    sys.exit(3)
if mode == "fail":
    time.sleep(60)             # must be stopped by the launcher, not waited for
if r == 0:
    print(json.dumps({"metric": "m", "value": 1.0, "n_gpus": w, "argv": sys.argv[1:]}), flush=True)
"""


def test_launch_ranks_spawns_world_and_forwards_rank0(tmp_path, capsys):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    rc = bench.launch_ranks(3, ["ok", "--steps", "2"], script=str(script))
    assert rc == 0
    lines = [l for l in capsys.readouterr().out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    row = json.loads(lines[0])
    assert row["n_gpus"] == 3 and row["argv"] == ["ok", "--steps", "2"]


def test_launch_ranks_stops_the_others_when_a_rank_fails(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    t0 = time.time()
    rc = bench.launch_ranks(2, ["fail"], script=str(script))
    assert rc == 3
    assert time.time() - t0 < 30


def test_launch_ranks_rejects_a_wrong_rank_count(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT.replace('"n_gpus": w', '"n_gpus": 1'))
    assert bench.launch_ranks(2, ["ok"], script=str(script)) == 1


def test_world_size_must_equal_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 1" in p.stderr


def test_gpus_n_parent_imports_no_package(tmp_path):
    """The --gpus N parent spawns before importing the package (which loads the HIP library):
    bench.py's module level holds no package import."""
    assert bench.pkg is None
