"""The culled row-sum task table of orient_desc_kernel (slam_framework_amd/csrc/orient_tasks.inc,
tools/gen_rs_tasks.py) covers every (window row, column) whose row sum a descriptor sample can
read: the kernel's own sample arithmetic (f32 rotation, round-half-even through the 1.5 * 2^23
magic add, rows sy - 3 .. sy + 3 of column sx) swept over angles, plus the regenerated table
matching the committed one."""
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "slam_framework_amd", "csrc")


def _pattern():
    src = open(os.path.join(CSRC, "orb_pattern.inc")).read()
    nums = [int(v) for v in re.findall(r"-?\d+", src.split("*/", 1)[1])]
    return np.array(nums[:1024], np.float32).reshape(512, 2)


def _tasks():
    src = open(os.path.join(CSRC, "orient_tasks.inc")).read()
    body = src.split("{", 1)[1].split("}", 1)[0]
    ent = [int(v, 16) for v in re.findall(r"0x[0-9a-f]+", body)]
    return {(e & 0xff, e >> 8) for e in ent if e != 0xffff}


def test_task_table_covers_every_sample_window():
    P = _pattern()
    tasks = _tasks()
    rng = np.random.default_rng(1)
    ang = np.concatenate([np.linspace(0, 360, 3601, dtype=np.float32),
                          rng.uniform(0, 360, 4000).astype(np.float32)])
    rad = (ang * np.float32(np.pi / 180.0)).astype(np.float32)
    s, c = np.sin(rad).astype(np.float32), np.cos(rad).astype(np.float32)
    px, py = P[:, 0][None, :], P[:, 1][None, :]
    magic = np.float32(12582912.0)
    sy = ((px * s[:, None] + py * c[:, None]).astype(np.float32) + magic) - magic
    sx = ((px * c[:, None] - py * s[:, None]).astype(np.float32) + magic) - magic
    pts = np.unique(np.stack([sx.ravel(), sy.ravel()], 1).astype(int), axis=0)
    assert np.abs(pts).max() <= 18
    need = {((y + d + 21) // 2, (x + 18) // 4) for x, y in pts.tolist() for d in range(-3, 4)}
    assert need <= tasks, sorted(need - tasks)[:8]
    assert len(tasks) <= 192  # three rounds of 64 lanes


def test_task_table_is_regenerated_identically(tmp_path):
    inc = os.path.join(CSRC, "orient_tasks.inc")
    before = open(inc).read()
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_rs_tasks.py")],
                          stdout=subprocess.DEVNULL)
    assert open(inc).read() == before
