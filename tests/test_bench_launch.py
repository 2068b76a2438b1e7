"""bench.py's multi-rank harness on CPU (no GPU, no kernel): `--gpus N` starts N ranks itself (torch.distributed.run as
a child process), every rank checks that the world it sees is N, the C3 set is LPT-sharded over the ranks and the
end-of-batch gather returns every utterance to rank 0 in order (`--dry-run`: gloo, placeholder codes)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_gpus2_starts_two_ranks_and_gathers_every_utterance():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["dry_run"] and line["n_gpus"] == 2
    c3 = line["c3_sharded"]
    assert c3["utterances"] == 16 and c3["gathered_utterances"] == c3["utterances"] and c3["gathered_in_order"]


def test_bench_refuses_a_world_that_is_not_gpus():
    # a launcher that started one rank for --gpus 2: the run must fail, not report a 1-GPU number as 2
    r = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0
    assert "launcher started 1 rank" in r.stderr
