"""Extract the DogBot link-state traces from the reference's Gazebo logs into
apf_quadruped_amd/data/gazebo_traces.npz.

Runs only where /root/reference exists (this container); the GPU box and the
tests read the committed .npz.  Data only: per recorded step the sim time, the
pose of every dogbot link (integers of 1e-5 m / rad, exactly as printed in the
log) and the base twist (1e-4 units), plus the link masses / inertial offsets and
the foot offset from the logged model insertion.

    python scripts/extract_gazebo_traces.py [/root/reference/DogBotV4/log]
"""
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from apf_quadruped_amd import traces  # noqa: E402


def main():
    logdir = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/DogBotV4/log"
    out, runs, const = {}, [], None
    for path in sorted(glob.glob(os.path.join(logdir, "*", "gzserver", "state.log"))):
        run = os.path.basename(os.path.dirname(os.path.dirname(path)))
        d = traces.parse_state_log(path)
        print(f"{run}: {len(d['t'])} steps", flush=True)
        if not len(d["t"]):
            continue
        runs.append(run)
        out[f"{run}/t"] = d["t"]
        out[f"{run}/pose"] = d["pose"].astype(np.int32)
        out[f"{run}/twist_base"] = d["twist_base"].astype(np.int32)
        if const is None:
            const = dict(mass=d["mass"], com=d["com"], foot=d["foot"])
    out.update(const)
    out["runs"] = np.array(runs)
    os.makedirs(os.path.dirname(traces.DATA), exist_ok=True)
    np.savez_compressed(traces.DATA, **out)
    print(traces.DATA, os.path.getsize(traces.DATA), "bytes")


if __name__ == "__main__":
    main()
