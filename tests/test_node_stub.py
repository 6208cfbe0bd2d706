"""The ROS1 node source (noetic-slam_amd/ros/tsdf_map_node.cpp) compiled and run off ROS: the
image has no ROS, so tests/ros_stubs stand in for roscpp and the four message types the node uses
(the node had never been compiled by anything).  Linked against the oracle library
(same C-ABI), the node's own main() runs; the stub spin() replays a DLIO-like topic stream into
its subscriptions, and the map the node writes at shutdown must equal integrating the same clouds
from the pose track (tests/test_host_replay.py's stream)."""
import os
import subprocess

import numpy as np
import pytest

import oracle
from conftest import REPO
from test_host_replay import oracle_voxels, read_bricks, topic_stream, write_topics
from tsdf_map import bricks_to_voxels

NODE = os.path.join(REPO, "noetic-slam_amd", "ros", "tsdf_map_node.cpp")
STUBS = os.path.join(REPO, "tests", "ros_stubs")


@pytest.fixture(scope="module")
def node_exe(tmp_path_factory):
    oracle.load()
    exe = tmp_path_factory.mktemp("node") / "tsdf_map_node"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", STUBS,
                           "-o", str(exe), NODE, "-L" + os.path.dirname(oracle.LIB_PATH),
                           "-ltsdf_oracle", "-Wl,-rpath," + os.path.dirname(oracle.LIB_PATH)])
    return str(exe)


@pytest.mark.parametrize("semantics", ["vdbfusion_f64", "vdbfusion", "voxblox", "voxblox_simple"])
def test_node_runs_topic_stream(tmp_path, sim, node_exe, semantics):
    recs, want = topic_stream(sim, tilt=0.5)
    write_topics(tmp_path / "in.topics", recs)
    out = tmp_path / "map.bricks"
    env = dict(os.environ, TSDF_STUB_STREAM=str(tmp_path / "in.topics"),
               TSDF_STUB_PARAMS="map_path=%s;min_range=0;semantics=%s;max_ray_length_m=1000%s" %
                                (out, semantics.split("_simple")[0],
                                 ";method=simple" if semantics.endswith("_simple") else ""))
    r = subprocess.run([node_exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "saved" in r.stderr
    got = bricks_to_voxels(*read_bricks(out))
    kw = dict(semantics=semantics.split("_simple")[0])
    if semantics.startswith("voxblox"):  # the node's voxblox defaults: merged (voxblox_ros')
        kw.update(max_range=1000.0, use_const_weight=False,
                  method="simple" if semantics.endswith("_simple") else "merged")
    ref = oracle_voxels(want, **kw)
    assert got[0].shape[0] > 1000
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)


def read_ply_soup(path):
    """The node's binary PLY triangle soup -> (3T, 3) float32 vertices."""
    data = open(path, "rb").read()
    head, _, body = data.partition(b"end_header\n")
    nv = int([ln for ln in head.split(b"\n") if ln.startswith(b"element vertex")][0].split()[2])
    return np.frombuffer(body[:12 * nv], np.float32).reshape(-1, 3)


def sector_volumes(n, yaw0, **kw):
    return [oracle.OracleTSDFVolume(0.05, 0.15, n_sectors=n, sector=k, sector_yaw0=yaw0, **kw)
            for k in range(n)]


def feed(vols, want):
    from test_host_replay import dlio_records
    for xyz, org in want:
        for v in vols:
            v.integrate_cloud(dlio_records(xyz).tobytes(), xyz.shape[0], 32, 0, org)


@pytest.mark.parametrize("num_gpus", [1, 2, 4])
def test_node_num_gpus_map_and_mesh(tmp_path, sim, node_exe, num_gpus):
    """~num_gpus > 1 gives the node N sector contexts (tsdf_create_sharded),
    feeds every cloud to all of them (tsdf_integrate_sectors) and border-reduces before writing:
    the map holds every observed brick once and equals the oracle's reduced sector fields bit for
    bit; against the single-volume field the weights are exact and |dS| <= 1e-5 m.  The mesh is
    written with the published Lorensen table (~mesh_table's default) -- for N > 1 through the
    sharded mesh (tsdf_extract_mesh_local), equal to the oracle's, triangle for triangle."""
    from test_border_local import sharded
    from test_distributed import tri_set
    from test_multigpu import emulated_reduce_host
    from tsdf_map import extract_mesh_local
    recs, want = topic_stream(sim, tilt=0.5)
    write_topics(tmp_path / "in.topics", recs)
    out, ply = tmp_path / "map.bricks", tmp_path / "mesh.ply"
    yaw0 = 0.7
    env = dict(os.environ, TSDF_STUB_STREAM=str(tmp_path / "in.topics"),
               TSDF_STUB_PARAMS="map_path=%s;mesh_path=%s;min_range=0;num_gpus=%d;sector_yaw0=%g"
                                % (out, ply, num_gpus, yaw0))
    r = subprocess.run([node_exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    coords, s, w = read_bricks(out)
    assert len({tuple(x) for x in coords.tolist()}) == coords.shape[0]  # each brick once
    got = bricks_to_voxels(coords, s, w)
    single = oracle_voxels(want)
    assert got[0].shape[0] > 1000
    assert np.array_equal(got[0], single[0]) and np.array_equal(got[2], single[2])
    assert np.max(np.abs(got[1] - single[1])) <= 1e-5
    mesh = read_ply_soup(ply)
    if num_gpus == 1:
        for a, b in zip(got, single):
            assert np.array_equal(a, b)
        o = oracle.OracleTSDFVolume(0.05, 0.15)
        o.import_bricks(coords, s, w)
        assert np.array_equal(mesh, o.extract_triangle_mesh(table="lorensen")[0])
        return
    vols = sector_volumes(num_gpus, yaw0)
    feed(vols, want)
    emulated_reduce_host(vols)
    ref = [v.export_bricks() for v in vols]
    keep = [(wk.reshape(len(ck), -1) > 0).any(1) for ck, _, wk in ref]
    want_vox = bricks_to_voxels(np.concatenate([ck[k] for (ck, _, _), k in zip(ref, keep)]),
                                np.concatenate([sk[k] for (_, sk, _), k in zip(ref, keep)]),
                                np.concatenate([wk[k] for (_, _, wk), k in zip(ref, keep)]))
    for a, b in zip(got, want_vox):
        assert np.array_equal(a.view(np.uint32) if a.dtype == np.float32 else a,
                              b.view(np.uint32) if b.dtype == np.float32 else b)
    shards = sharded(num_gpus, yaw0=yaw0)
    feed(shards, want)
    vm, _ = extract_mesh_local(shards, table="lorensen")
    assert mesh.shape[0] > 1000 and np.array_equal(tri_set(mesh), tri_set(vm))


@pytest.mark.gpu
@pytest.mark.parametrize("num_gpus", [2, 4])
def test_node_num_gpus_on_gpu(tmp_path, sim, num_gpus):
    """The node's own source linked to libtsdf_hip.so (noetic-slam_amd/lib/tsdf_map_node_offros,
    built by __graft_entry__.build()) with ~num_gpus sector contexts, all on GPU 0 here
    (~device_ids "0,0,..."; one per GPU on a node): the written map equals the oracle's reduced
    sector fields bit for bit (weights exact and |dS| <= 1e-5 m against the single volume), and
    the mesh equals the oracle's sharded Lorensen mesh triangle for triangle."""
    from test_border_local import sharded
    from test_distributed import tri_set
    from test_multigpu import emulated_reduce_host
    from tsdf_map import extract_mesh_local
    exe = os.path.join(REPO, "noetic-slam_amd", "lib", "tsdf_map_node_offros")
    assert os.path.exists(exe), "run __graft_entry__.build() first"
    recs, want = topic_stream(sim, tilt=0.5)
    write_topics(tmp_path / "in.topics", recs)
    out, ply = tmp_path / "map.bricks", tmp_path / "mesh.ply"
    yaw0 = 0.7
    env = dict(os.environ, TSDF_STUB_STREAM=str(tmp_path / "in.topics"),
               TSDF_STUB_PARAMS="map_path=%s;mesh_path=%s;min_range=0;num_gpus=%d;sector_yaw0=%g;"
                                "device_ids=%s" % (out, ply, num_gpus, yaw0,
                                                   ",".join(["0"] * num_gpus)))
    r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    assert "border reduce" in r.stderr
    coords, s, w = read_bricks(out)
    assert len({tuple(x) for x in coords.tolist()}) == coords.shape[0]
    got = bricks_to_voxels(coords, s, w)
    single = oracle_voxels(want)
    assert np.array_equal(got[0], single[0]) and np.array_equal(got[2], single[2])
    assert np.max(np.abs(got[1] - single[1])) <= 1e-5
    vols = sector_volumes(num_gpus, yaw0)
    feed(vols, want)
    emulated_reduce_host(vols)
    ref = [v.export_bricks() for v in vols]
    keep = [(wk.reshape(len(ck), -1) > 0).any(1) for ck, _, wk in ref]
    want_vox = bricks_to_voxels(np.concatenate([ck[k] for (ck, _, _), k in zip(ref, keep)]),
                                np.concatenate([sk[k] for (_, sk, _), k in zip(ref, keep)]),
                                np.concatenate([wk[k] for (_, _, wk), k in zip(ref, keep)]))
    assert np.array_equal(got[0], want_vox[0]) and np.array_equal(got[2], want_vox[2])
    assert np.array_equal(got[1].view(np.uint32), want_vox[1].view(np.uint32))
    shards = sharded(num_gpus, yaw0=yaw0)
    feed(shards, want)
    vm, _ = extract_mesh_local(shards, table="lorensen")
    mesh = read_ply_soup(ply)
    assert mesh.shape[0] > 1000 and np.array_equal(tri_set(mesh), tri_set(vm))


def _write_with(path, recs, extra):
    """write_topics plus bare control records: extra = {index: b"S" | b"X"} placed before recs[index]
    ('S' calls ~save_map, 'X' ends the process there: ros_stubs/README.md)."""
    import struct
    from test_host_replay import dlio_records
    with open(path, "wb") as f:
        f.write(b"TSDFSTR2")
        for i, (kind, t, v) in enumerate(recs + [("END", 0, None)]):
            if i in extra:
                f.write(extra[i] + struct.pack("<q", 0))
            if kind == "P":
                f.write(b"P" + struct.pack("<q3d4d", t, *v[0], *v[1]))
            elif kind == "C":
                rec = dlio_records(v)
                f.write(b"C" + struct.pack("<qQIIi", t, rec.shape[0], 32, 0, 0) + rec.tobytes())


def _integrated(stderr, what):
    """The node's count of integrated clouds at its last checkpoint / save_map call."""
    import re
    pat = r"checkpoint after \d+ clouds \((\d+) integrated\)" if what == "checkpoint" else \
        r"save_map: (\d+) clouds integrated"
    got = re.findall(pat, stderr)
    assert got, stderr
    return int(got[-1])


def _check_map(path, want_scans, num_gpus):
    coords, s, w = read_bricks(path)
    assert len({tuple(x) for x in coords.tolist()}) == coords.shape[0]  # each brick once
    got = bricks_to_voxels(coords, s, w)
    single = oracle_voxels(want_scans)
    assert got[0].shape[0] > 500
    assert np.array_equal(got[0], single[0]) and np.array_equal(got[2], single[2])
    if num_gpus == 1:
        assert np.array_equal(got[1].view(np.uint32), single[1].view(np.uint32))
    else:
        assert np.max(np.abs(got[1] - single[1])) <= 1e-5
    return coords, s, w


@pytest.mark.parametrize("num_gpus", [1, 2])
def test_node_checkpoint_survives_a_crash(tmp_path, sim, node_exe, num_gpus):
    """~save_every_n_clouds writes the map while the node runs (dliomapping's
    every-999 dump, dliomapping.cpp:72-80).  The process then dies without its shutdown save (the
    stub's 'X' record): the file on disk is the last checkpoint, and it equals the map of the clouds
    integrated by then (bit for bit on one context; with two GPUs the reduced map: weights exact,
    |dS| <= 1e-5 m against the single volume)."""
    recs, want = topic_stream(sim, tilt=0.5)
    cl = [i for i, r in enumerate(recs) if r[0] == "C"]
    out = tmp_path / "map.bricks"
    # die right after the 5th cloud record (the checkpoint after the 3rd has been written)
    _write_with(tmp_path / "in.topics", recs, {cl[4] + 1: b"X"})
    env = dict(os.environ, TSDF_STUB_STREAM=str(tmp_path / "in.topics"),
               TSDF_STUB_PARAMS="map_path=%s;min_range=0;num_gpus=%d;save_every_n_clouds=3"
                                % (out, num_gpus))
    r = subprocess.run([node_exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, r.stderr  # the crash, not a clean exit
    m = _integrated(r.stderr, "checkpoint")
    assert 1 <= m < len(want)
    assert not os.path.exists(str(out) + ".tmp")
    _check_map(out, want[:m], num_gpus)


def test_node_save_service_and_failed_reduce(tmp_path, sim, node_exe):
    """VERDICT r5 #5 / ADVICE r5: with two GPUs and the border reduce failing (the oracle's
    injected failure, an aborted transaction: every context unchanged), the node retries once and
    then merges the contexts' bricks on the host.  The ~save_map service (std_srvs/Trigger, DLIO's
    save_pcd in spirit, map.cc:81-111) called mid-stream writes that map and its mesh; a crash
    right after leaves them on disk.  The map equals the single volume (weights exact, |dS| <= 1e-5
    m) and the mesh is the published-table mesh of that map, triangle for triangle."""
    from test_distributed import tri_set
    recs, want = topic_stream(sim, tilt=0.5)
    cl = [i for i, r in enumerate(recs) if r[0] == "C"]
    out, ply = tmp_path / "map.bricks", tmp_path / "mesh.ply"
    _write_with(tmp_path / "in.topics", recs, {cl[4] + 1: b"S", cl[4] + 2: b"X"})
    env = dict(os.environ, TSDF_STUB_STREAM=str(tmp_path / "in.topics"), TSDF_ORACLE_REDUCE_FAIL="2",
               TSDF_STUB_PARAMS="map_path=%s;mesh_path=%s;min_range=0;num_gpus=2;"
                                "save_every_n_clouds=0" % (out, ply))
    r = subprocess.run([node_exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, r.stderr
    assert "retrying" in r.stderr and "host-merged" in r.stderr
    assert "service save_map: success" in r.stderr
    m = _integrated(r.stderr, "save_map")
    assert 1 <= m <= len(want)
    coords, s, w = _check_map(out, want[:m], 2)
    o = oracle.OracleTSDFVolume(0.05, 0.15)
    o.import_bricks(coords, s.reshape(-1, 8, 8, 8), w.reshape(-1, 8, 8, 8))
    mesh = read_ply_soup(ply)
    assert mesh.shape[0] > 1000
    assert np.array_equal(tri_set(mesh), tri_set(o.extract_triangle_mesh(table="lorensen")[0]))


def test_node_shutdown_save_after_failed_reduce(tmp_path, sim, node_exe):
    """The shutdown write with a reduce that fails twice: the map is still written (host-merged),
    not lost (round 5 returned before writing anything)."""
    recs, want = topic_stream(sim, tilt=0.5)
    write_topics(tmp_path / "in.topics", recs)
    out = tmp_path / "map.bricks"
    env = dict(os.environ, TSDF_STUB_STREAM=str(tmp_path / "in.topics"), TSDF_ORACLE_REDUCE_FAIL="2",
               TSDF_STUB_PARAMS="map_path=%s;min_range=0;num_gpus=2;save_every_n_clouds=0" % out)
    r = subprocess.run([node_exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "host-merged" in r.stderr
    _check_map(out, want, 2)


def test_node_failed_reduce_voxblox_weight_cap(tmp_path, sim, node_exe):
    """The host merge after a failed reduce follows the reduce's own rule, Voxblox's max_weight cap
    included: two Voxblox (Merged, 1/z^2) sector contexts with max_weight = 2, the reduce failing
    twice -- the node's host-merged map equals the oracle's sector fields after a reduce that ran,
    bit for bit (rank 0's bricks first, then rank 1's merged into them, W capped at 2)."""
    from test_multigpu import emulated_reduce_host
    recs, want = topic_stream(sim, tilt=0.5)
    write_topics(tmp_path / "in.topics", recs)
    out = tmp_path / "map.bricks"
    env = dict(os.environ, TSDF_STUB_STREAM=str(tmp_path / "in.topics"), TSDF_ORACLE_REDUCE_FAIL="2",
               TSDF_STUB_PARAMS="map_path=%s;min_range=0;num_gpus=2;save_every_n_clouds=0;"
                                "semantics=voxblox;max_ray_length_m=1000;max_weight=2" % out)
    r = subprocess.run([node_exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "host-merged" in r.stderr
    coords, s, w = read_bricks(out)
    assert len({tuple(x) for x in coords.tolist()}) == coords.shape[0]  # each brick once
    got = bricks_to_voxels(coords, s, w)
    vols = sector_volumes(2, 0.0, semantics="voxblox", max_range=1000.0, use_const_weight=False,
                          method="merged", max_weight=2.0)
    feed(vols, want)
    emulated_reduce_host(vols)
    ref = [v.export_bricks() for v in vols]
    keep = [(wk.reshape(len(ck), -1) > 0).any(1) for ck, _, wk in ref]
    want_vox = bricks_to_voxels(np.concatenate([ck[k] for (ck, _, _), k in zip(ref, keep)]),
                                np.concatenate([sk[k] for (_, sk, _), k in zip(ref, keep)]),
                                np.concatenate([wk[k] for (_, _, wk), k in zip(ref, keep)]))
    assert got[0].shape[0] > 1000 and np.any(got[2] == 2.0)  # the cap binds somewhere
    for a, b in zip(got, want_vox):
        assert np.array_equal(a.view(np.uint32) if a.dtype == np.float32 else a,
                              b.view(np.uint32) if b.dtype == np.float32 else b)
