"""bench.py --gpus N without a launcher starts N ranks itself (VERDICT r3 'next' 2); with a launcher, WORLD_SIZE must
agree with --gpus.  CPU only: the reconciliation table and the child launcher on a stand-in script."""
import importlib.util
import os
import sys

import pytest

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_resolve_world_table():
    b = _bench()
    assert b.resolve_world(1, {}) == ("run", 1)
    assert b.resolve_world(8, {}) == ("spawn", 8)
    assert b.resolve_world(4, {"WORLD_SIZE": "4"}) == ("run", 4)
    assert b.resolve_world(1, {"WORLD_SIZE": "1"}) == ("run", 1)
    with pytest.raises(SystemExit):
        b.resolve_world(2, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        b.resolve_world(1, {"WORLD_SIZE": "2"})


def test_launch_ranks_environment(tmp_path):
    """Each child sees its RANK / LOCAL_RANK, the common WORLD_SIZE and a 127.0.0.1 rendezvous; exit 0 overall."""
    b = _bench()
    script = tmp_path / "rank.py"
    out = tmp_path / "out"
    out.mkdir()
    script.write_text("import os, sys\n"
                      "e = os.environ\n"
                      "open(os.path.join(sys.argv[1], e['RANK']), 'w').write("
                      "' '.join([e['LOCAL_RANK'], e['WORLD_SIZE'], e['MASTER_ADDR'], e['MASTER_PORT']]))\n")
    rc, rcs = b.launch_ranks(3, str(script), [str(out)])
    assert rc == 0 and rcs == [0, 0, 0]
    seen = {int(f): open(out / f).read().split() for f in os.listdir(out)}
    assert sorted(seen) == [0, 1, 2]
    ports = {v[3] for v in seen.values()}
    assert len(ports) == 1
    for r, (local, world, addr, _) in seen.items():
        assert int(local) == r and world == "3" and addr == "127.0.0.1"


def test_launch_ranks_failure_stops_the_rest(tmp_path):
    """A failing rank ends the job: the other ranks (blocked, as in a collective) are terminated and the worst status
    comes back."""
    b = _bench()
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1':\n"
                      "    sys.exit(3)\n"
                      "time.sleep(60)\n")
    rc, rcs = b.launch_ranks(2, str(script), [])
    assert rc != 0 and rcs[1] == 3


def test_bench_spawns_without_launcher(tmp_path):
    """The real entry point: `python bench.py --gpus 2` with no WORLD_SIZE takes the spawn path before importing torch
    (checked by running main() with launch_ranks replaced)."""
    b = _bench()
    calls = []
    b.launch_ranks = lambda n, script, argv: (calls.append((n, script, argv)) or (0, [0] * n))
    saved = sys.argv, os.environ.pop("WORLD_SIZE", None)
    sys.argv = ["bench.py", "--gpus", "2", "--steps", "3"]
    try:
        with pytest.raises(SystemExit) as e:
            b.main()
        assert e.value.code == 0
    finally:
        sys.argv = saved[0]
        if saved[1] is not None:
            os.environ["WORLD_SIZE"] = saved[1]
    assert calls and calls[0][0] == 2 and calls[0][2] == ["--gpus", "2", "--steps", "3"]
