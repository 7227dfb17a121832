"""CPU tests of bench.py's rank launcher: ``python bench.py --gpus N`` without a launcher
starts N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, nothing
touching the GPU in the parent); under torchrun (WORLD_SIZE present) it runs as a rank."""
import os
import sys
import time

import bench


def test_launch_plan_without_launcher():
    env = {"PATH": os.environ.get("PATH", "")}
    plan = bench.launch_plan(4, env)
    assert [e["RANK"] for e in plan] == ["0", "1", "2", "3"]
    assert all(e["LOCAL_RANK"] == e["RANK"] and e["WORLD_SIZE"] == "4" for e in plan)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" for e in plan)
    assert len({e["MASTER_PORT"] for e in plan}) == 1 and int(plan[0]["MASTER_PORT"]) > 0


def test_launch_plan_is_none_under_a_launcher_or_one_gpu():
    assert bench.launch_plan(8, {"WORLD_SIZE": "8", "RANK": "3"}) is None
    assert bench.launch_plan(1, {}) is None
    assert bench.launch_plan(2, {"MASTER_PORT": "29511"})[1]["MASTER_PORT"] == "29511"


def test_run_ranks_collects_every_rank(tmp_path):
    out = tmp_path / "ranks"
    out.mkdir()
    script = tmp_path / "rank.py"
    script.write_text("import os, sys\n"
                      f"open(os.path.join({str(out)!r}, os.environ['RANK']), 'w').write(os.environ['WORLD_SIZE'])\n")
    rc = bench.run_ranks(bench.launch_plan(3, dict(os.environ, PYTHONPATH="")), [], script=str(script))
    assert rc == 0
    assert sorted(os.listdir(out)) == ["0", "1", "2"]
    assert all((out / r).read_text() == "3" for r in ("0", "1", "2"))


def test_run_ranks_stops_the_others_when_a_rank_fails(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1':\n    sys.exit(3)\n"
                      "time.sleep(120)\n")
    t0 = time.time()
    rc = bench.run_ranks(bench.launch_plan(2, dict(os.environ)), [], script=str(script))
    assert rc == 3 and time.time() - t0 < 60
