"""A/B of tile-config tables inside one process: run bench.py's main() with
rrin_amd.engine.H8_TUNED patched by JSON overrides.

usage: python tools/bench_ab.py '{"(32,32,0)": 8}' -- [bench.py args]"""
import ast
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rrin_amd import _lib, engine  # noqa: E402

over = json.loads(sys.argv[1])
rest = sys.argv[sys.argv.index("--") + 1:] if "--" in sys.argv else []
prec = _lib.PREC_F16 if "fp16" in rest else _lib.PREC_F16X3
for k, v in over.items():
    engine.H8_TUNED[prec][tuple(ast.literal_eval(k))] = int(v)
sys.argv = ["bench.py"] + rest
import bench  # noqa: E402

print("overrides", over, file=sys.stderr)
bench.main()
