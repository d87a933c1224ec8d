#!/usr/bin/env python3
"""Per-phase kernel durations of the driver's default bench command from its rocprofv3 kernel trace.

The default command (``bench.py --gpus 1 --steps 20 --warmup 5``) launches episode_fast_kernel for
the configs[1] warm-up (episodes 0-4), the timed region (5-24) and the epsilon-schedule
continuation (25-999, value_at_eps), then episode_sq16_kernel for the configs[2] secondary
(2 warm-up + 10 timed).  rocprofv3 --stats averages over every launch, so its configs[1] average
is mostly the continuation (lower epsilon, slower episodes); this script splits the trace by launch
index so each phase's average can be set beside the HIP-event kernel_ms of the bench line.  With
chained launches (the line's launch.launches: [first episode, episodes] per launch) each launch's
duration is split evenly over its episodes; the phase averages are per episode.

    python scripts/summarize_trace.py gpurun_out/r05/prof_c2/c2_kernel_trace.csv gpurun_out/r05/c2.json \
        > profiles/r05_bench_kernel_phases.json
"""
import csv
import json
import sys


def durations(path, key):
    rows = [r for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in rows]  # us


def avg(xs):
    return sum(xs) / len(xs) if xs else None


def per_episode(fast, line):
    """Per-episode kernel time in episode order: chained launches (line["launch"]["launches"] =
    [first episode, episodes] in launch order) split evenly over their episodes."""
    launches = (line.get("launch") or {}).get("launches")
    if not launches:
        return fast
    assert len(launches) == len(fast), (len(launches), len(fast))
    out = []
    for (first, n), d in zip(launches, fast):
        assert first == len(out), (first, len(out))
        out += [d / n] * n
    return out


def main(trace, line_path):
    line = json.loads(open(line_path).read().strip().splitlines()[-1])
    w, k = line["warmup"], line["steps"]
    launch_us = durations(trace, "episode_fast_kernel")
    fast = per_episode(launch_us, line)
    out = {"trace": trace, "line": line_path, "episode_fast_kernel": {
        "launches": len(launch_us), "episodes": len(fast), "all_launches_us": avg(launch_us),
        "all_episodes_us": avg(fast),
        "timed_region": {"episodes": [w, w + k], "avg_us": avg(fast[w:w + k]),
                         "line_kernel_ms": line["roofline"]["kernel_ms"]}}}
    ve = line.get("value_at_eps")
    if ve:
        wins = []
        for win in ve["windows"]:
            a = win["first_episode"]
            wins.append({"episodes": [a, a + win["episodes"]], "epsilon": win["epsilon"],
                         "avg_us": avg(fast[a:a + win["episodes"]]), "line_kernel_ms": win["kernel_ms"]})
        out["episode_fast_kernel"]["epsilon_windows"] = wins
        c = ve["continuation"]
        a = c["first_episode"]
        out["episode_fast_kernel"]["continuation"] = {"episodes": [a, a + c["episodes"]],
                                                      "avg_us": avg(fast[a:a + c["episodes"]])}
    sec = line.get("secondary")
    if sec and "roofline" in sec:
        sq = durations(trace, "episode_sq16_kernel")
        sw, sk = sec["warmup"], sec["steps"]
        out["episode_sq16_kernel"] = {"launches": len(sq), "all_launches_us": avg(sq),
                                      "timed_region": {"episodes": [sw, sw + sk], "avg_us": avg(sq[sw:sw + sk]),
                                                       "line_kernel_ms": sec["roofline"]["kernel_ms"]}}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:3])
