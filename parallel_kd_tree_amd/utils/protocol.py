"""Reference CLI protocol in Python (Utility.cpp:66-124), byte-compatible with the C++
executables: READY / stdin seed or argv SEED DIM_POINTS NUM_POINTS / ID-DISTANCE lines /
[elapsed time] / DONE. Floats are printed like std::ostream (%g, 6 significant digits)."""
from __future__ import annotations

import sys
from typing import List, Tuple


def validate_input(seed: int, dim: int, n: int) -> None:
    err = sys.stderr
    if seed == 0:
        print("Warning: default value 0 used as seed.", file=err, flush=True)
    if seed < 0:
        print("Seed has to be larger than 0!", file=err, flush=True)
        sys.exit(1)
    if dim <= 0:
        print("Dimension has to be larger than 0!", file=err, flush=True)
        sys.exit(1)
    if n <= 0:
        print("Number of points has to be larger than 0!", file=err, flush=True)
        sys.exit(1)
    print(f"\tUsing seed {seed}", file=err)
    print(f"\tUsing point dimensions {dim}", file=err)
    print(f"\tUsing number of points {n}\n", file=err, flush=True)


def specify_problem_stdin() -> Tuple[int, int, int]:
    print("READY", flush=True)
    print("Specify seed ", end="", file=sys.stderr, flush=True)
    seed = int(sys.stdin.readline().split()[0])
    validate_input(seed, 128, 500000)
    return seed, 128, 500000


def specify_problem_argv(argv0: str, args: List[str]) -> Tuple[int, int, int]:
    if len(args) != 3:
        print(f"Usage: {argv0} SEED DIM_POINTS  NUM_POINTS", file=sys.stderr, flush=True)
        sys.exit(1)
    print("READY", flush=True)
    seed, dim, n = (int(a) for a in args)
    validate_input(seed, dim, n)
    return seed, dim, n


def fmt_float(v: float) -> str:
    return "%g" % v


def result_line(qid: int, distance: float) -> str:
    return f"ID: {qid} \t DISTANCE: {fmt_float(distance)}"
