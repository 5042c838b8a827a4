"""A/B of the replay gather's words-per-thread (DDQ_GATHER_WPT, read once per
process): prints bench.gather_stress() for the value in the environment.

usage: DDQ_GATHER_WPT=8 python tools/gpu/gather_ab.py"""
import json
import os
import sys

R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, os.path.join(R, "distributed-deep-q_amd"))
sys.path.insert(0, R)
import bench  # noqa: E402

r = bench.gather_stress()
print(os.environ.get("DDQ_GATHER_WPT", "4"),
      json.dumps([(x["n"], x["gather_us"], x["gather_GBps"]) for x in r["launches"]]), flush=True)
