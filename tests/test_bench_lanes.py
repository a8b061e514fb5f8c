"""bench.py's lanes runner (CPU): n batches over concurrent host threads, as
the SttEngine's parallel_requests batchers run them (DESIGN.md "lanes")."""
import os
import random
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("n,lanes", [(6, 2), (7, 2), (6, 3), (1, 4), (5, 1), (0, 2)])
def test_every_batch_once_in_order(n, lanes):
    lock = threading.Lock()
    count = [0]
    rng = random.Random(n * 10 + lanes)
    delays = [rng.uniform(0.0, 0.01) for _ in range(n)]

    def step(lane):
        with lock:
            k = count[0]
            count[0] += 1
        time.sleep(delays[k])
        return (k, lane)

    out = bench.run_lanes(n, lanes, step)
    assert len(out) == n and count[0] == n
    # results come back in batch order: batch i is the i-th batch handed out
    assert sorted(k for k, _ in out) == list(range(n))
    assert all(0 <= lane < max(1, lanes) for _, lane in out)


def test_lanes_run_concurrently():
    inside, peak = [0], [0]
    lock = threading.Lock()

    def step(lane):
        with lock:
            inside[0] += 1
            peak[0] = max(peak[0], inside[0])
        time.sleep(0.05)
        with lock:
            inside[0] -= 1
        return lane

    out = bench.run_lanes(4, 2, step)
    assert peak[0] == 2 and sorted(set(out)) == [0, 1]


def test_error_stops_lanes_and_is_raised():
    calls = [0]
    lock = threading.Lock()

    def step(lane):
        with lock:
            calls[0] += 1
            k = calls[0]
        if k == 2:
            raise RuntimeError("mwx_full_batch rc=-1")
        time.sleep(0.01)
        return k

    with pytest.raises(RuntimeError, match="rc=-1"):
        bench.run_lanes(50, 2, step)
    assert calls[0] < 50


def test_service_leg_rides_only_on_the_full_default_run():
    from types import SimpleNamespace
    base = dict(no_service_leg=False, no_cpu_baseline=False, service_defaults=False,
                arch="large-v3", beam=0, fp8=False, rich=False, decode_steps=220,
                clip_seconds=30.0, host_input=False)
    assert bench.is_headline_config(SimpleNamespace(**base))
    for k, v in [("no_service_leg", True), ("no_cpu_baseline", True), ("service_defaults", True),
                 ("arch", "base"), ("beam", 5), ("fp8", True), ("rich", True),
                 ("decode_steps", 0), ("clip_seconds", 600.0), ("host_input", True)]:
        assert not bench.is_headline_config(SimpleNamespace(**{**base, k: v})), k
