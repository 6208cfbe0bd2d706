"""Extract the Ouster beam-intrinsics fixtures used by the synthetic scan generator.

Reads two sensor-metadata JSONs that ship with the reference's Ouster SDK tests (data files, not
code) and writes their beam angles to tests/golden/ouster_beams.json, so the generator runs on the
GPU box where /root/reference does not exist.  Run once in the build container:

    python tests/golden/make_beams.py

Sources:
  OS-1-128 1024x10:  src/ouster/ouster-sdk/tests/metadata/2_4_0_os-992146000760-128.json
  OS-1-128 2048x10:  src/ouster/ouster-sdk/tests/metadata/2_0_0_os1-992008000494-128_col_win_legacy.json
"""
import json
import os

REF = "/root/reference/src/ouster/ouster-sdk/tests/metadata"
HERE = os.path.dirname(os.path.abspath(__file__))


def _extract(path, columns):
    d = json.load(open(path))
    bi = d.get("beam_intrinsics", d)
    return {
        "source": "reference:" + os.path.relpath(path, "/root/reference"),
        "columns_per_frame": columns,
        "pixels_per_column": len(bi["beam_altitude_angles"]),
        "beam_altitude_angles": bi["beam_altitude_angles"],
        "beam_azimuth_angles": bi["beam_azimuth_angles"],
        "lidar_origin_to_beam_origin_mm": bi["lidar_origin_to_beam_origin_mm"],
    }


def main():
    out = {
        "os1_128_1024": _extract(os.path.join(REF, "2_4_0_os-992146000760-128.json"), 1024),
        "os1_128_2048": _extract(
            os.path.join(REF, "2_0_0_os1-992008000494-128_col_win_legacy.json"), 2048),
    }
    with open(os.path.join(HERE, "ouster_beams.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
