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


def test_pmc_summary_selection_takes_the_newest_matching_profile(tmp_path):
    """bench.py's roofline traffic comes from the newest PMC summary of the SAME code: the
    algorithmic bytes AND the date-iterations per step must match; uppercase run letters
    (used after a..z) sort after lowercase ones; profiles/EVIDENCE.json wins when it matches."""
    import json
    pdir = tmp_path / "profiles"
    pdir.mkdir()

    def put(tag, it_bytes, iters, hbm):
        (pdir / f"{tag}_pmc_summary.json").write_text(json.dumps(
            {"admm_iterations_per_step": iters,
             "kernels": {"k_admm_gcap": {"algorithmic_bytes_per_admm_iteration": float(it_bytes),
                                         "hbm_bytes_per_admm_iteration": hbm}}}))
    put("r03v", 541252, 61737, 1.0)
    put("r03S", 541252, 61737, 2.0)       # newer than r03v (uppercase letters follow z)
    put("r03T", 541252, 70000, 3.0)       # newer, but other iterations: another code state
    put("r02j", 541252, 61737, 4.0)
    sel = bench.select_pmc_summary("k_admm_gcap", 541252, 61737, root=str(tmp_path))
    assert sel is not None and sel[0].endswith("r03S_pmc_summary.json") and sel[1]["kernels"]["k_admm_gcap"][
        "hbm_bytes_per_admm_iteration"] == 2.0
    assert bench.select_pmc_summary("k_admm_gcap", 541252, 12345, root=str(tmp_path)) is None
    put("r04a", 541252, 61737, 5.0)
    assert bench.select_pmc_summary("k_admm_gcap", 541252, 61737, root=str(tmp_path))[0].endswith("r04a_pmc_summary.json")
    (pdir / "EVIDENCE.json").write_text(json.dumps({"pmc_summary": "r03v_pmc_summary.json"}))
    assert bench.select_pmc_summary("k_admm_gcap", 541252, 61737, root=str(tmp_path))[0].endswith("r03v_pmc_summary.json")
    assert sorted(["r03a", "r03S", "r03z", "r04a", "r03A"], key=bench.profile_order) == \
        ["r03a", "r03z", "r03A", "r03S", "r04a"]
