"""Per-GPU host-core split of the stream worker pools (VERDICT r4 item 7,
SURVEY.md s8(e) "one worker pool per GPU, cores split per GPU, NUMA-local"),
on fake sysfs topologies -- no GPU: the split is computed by the library's own
C++ (numa_affinity.hip split_worker_cpus) through hjd_debug_worker_cpus.

The 8-GPU node of the bench (2 sockets, 2 NUMA nodes, 4 GPUs per node) gives
each GPU a disjoint quarter of its node's CPUs."""
import os

import pytest

hjd = pytest.importorskip("ocljpegdecoder_amd")

GPUS8 = ["0000:05:00.0", "0000:15:00.0", "0000:65:00.0", "0000:75:00.0",
         "0000:85:00.0", "0000:95:00.0", "0000:E5:00.0", "0000:F5:00.0"]


def _tree(tmp_path, nodes, gpu_node):
    """nodes: {node: cpulist string}; gpu_node: {bus id: node}."""
    root = tmp_path / "fake"
    for n, cl in nodes.items():
        d = root / "sys" / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cl + "\n")
    for bus, n in gpu_node.items():
        d = root / "sys" / "bus" / "pci" / "devices" / bus.lower()
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{n}\n")
    return str(root)


def _expand(cl):
    out = []
    for part in cl.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def test_two_socket_eight_gpus(tmp_path):
    nodes = {0: "0-63,128-191", 1: "64-127,192-255"}
    root = _tree(tmp_path, nodes, {g: (0 if i < 4 else 1) for i, g in enumerate(GPUS8)})
    sets = [hjd.worker_cpus(g, GPUS8, root) for g in GPUS8]
    for i, s in enumerate(sets):
        assert len(s) == 32, (i, len(s))
        assert set(s) <= set(_expand(nodes[0 if i < 4 else 1]))        # NUMA-local
    for node in (0, 1):
        got = [c for s in sets[4 * node:4 * node + 4] for c in s]
        assert sorted(got) == _expand(nodes[node])                       # the node split exactly once
    # bus ids in another case / order give the same split
    rev = [g.lower() for g in reversed(GPUS8)]
    assert [hjd.worker_cpus(g, rev, root) for g in GPUS8] == sets


def test_uneven_and_degenerate_topologies(tmp_path):
    # 3 GPUs on a 10-CPU node: slices of 4, 3, 3; a lone GPU on node 1 takes the whole node
    nodes = {0: "0-9", 1: "10-13"}
    gpus = GPUS8[:4]
    root = _tree(tmp_path, nodes, {gpus[0]: 0, gpus[1]: 0, gpus[2]: 0, gpus[3]: 1})
    assert [hjd.worker_cpus(g, gpus, root) for g in gpus] == [[0, 1, 2, 3], [4, 5, 6], [7, 8, 9], [10, 11, 12, 13]]
    # a process that sees only its own GPU (one visible device) keeps the node
    assert hjd.worker_cpus(gpus[1], [gpus[1]], root) == list(range(10))
    # fewer CPUs than GPUs on a node: they share it
    root2 = _tree(tmp_path / "b", {0: "0-2"}, {g: 0 for g in gpus})
    assert all(hjd.worker_cpus(g, gpus, root2) == [0, 1, 2] for g in gpus)
    # unknown NUMA node (-1) or no sysfs entry: no binding
    root3 = _tree(tmp_path / "c", {0: "0-7"}, {gpus[0]: -1})
    assert hjd.worker_cpus(gpus[0], gpus[:1], root3) == []
    assert hjd.worker_cpus("0000:aa:00.0", gpus, root3) == []


def test_allowed_cpus_intersection(tmp_path):
    """only_allowed keeps the CPUs this process may run on (container cpusets)."""
    allowed = sorted(os.sched_getaffinity(0))
    hi = max(allowed)
    root = _tree(tmp_path, {0: f"0-{hi + 64}"}, {GPUS8[0]: 0})
    assert hjd.worker_cpus(GPUS8[0], GPUS8[:1], root, only_allowed=True) == allowed
    assert len(hjd.worker_cpus(GPUS8[0], GPUS8[:1], root)) == hi + 65


def test_stream_threads_eight_gpu_node(tmp_path):
    """bench.py config 5's per-GPU host worker count on the 8-GPU node's
    topology (2 NUMA nodes x 128 logical CPUs, 4 GPUs each): with no cgroup
    quota every rank uses its whole 32-CPU slice (SMT siblings included); a
    quota splits over the ranks first; a one-GPU 16-CPU box keeps 16."""
    nodes = {0: "0-63,128-191", 1: "64-127,192-255"}
    root = _tree(tmp_path, nodes, {g: (0 if i < 4 else 1) for i, g in enumerate(GPUS8)})
    slices = [len(hjd.worker_cpus(g, GPUS8, root)) for g in GPUS8]
    assert slices == [32] * 8
    assert [hjd.stream_worker_threads(256, 8, n) for n in slices] == [32] * 8      # no quota
    assert [hjd.stream_worker_threads(128, 8, n) for n in slices] == [16] * 8      # quota 128 CPUs
    assert hjd.stream_worker_threads(16, 1, 128) == 16                             # the one-GPU box
    assert hjd.stream_worker_threads(256, 8, 0) == 32                              # unknown topology


def _cgroup_tree(tmp_path, self_cgroup, files):
    root = tmp_path / "cg"
    (root / "proc" / "self").mkdir(parents=True)
    (root / "proc" / "self" / "cgroup").write_text(self_cgroup)
    for rel, text in files.items():
        f = root / rel
        f.parent.mkdir(parents=True, exist_ok=True)
        f.write_text(text)
    return str(root)


def test_cpu_share_cgroup_versions(tmp_path):
    """hjd_host_cpu_share's quota on fake trees: v2 at the root and nested (an
    ancestor's smaller limit wins), v1 cpu,cpuacct, and no quota at all."""
    aff = len(os.sched_getaffinity(0))
    cases = [
        ("0::/\n", {"sys/fs/cgroup/cpu.max": "300000 100000\n"}, 3),
        ("0::/a/b\n", {"sys/fs/cgroup/a/b/cpu.max": "max 100000\n", "sys/fs/cgroup/a/cpu.max": "250000 100000\n"}, 3),
        ("0::/a/b\n", {"sys/fs/cgroup/a/b/cpu.max": "100000 100000\n", "sys/fs/cgroup/a/cpu.max": "800000 100000\n"}, 1),
        ("12:cpu,cpuacct:/docker/x\n3:memory:/docker/x\n",
         {"sys/fs/cgroup/cpu,cpuacct/docker/x/cpu.cfs_quota_us": "200000\n",
          "sys/fs/cgroup/cpu,cpuacct/docker/x/cpu.cfs_period_us": "100000\n"}, 2),
        ("12:cpu,cpuacct:/\n", {"sys/fs/cgroup/cpu,cpuacct/cpu.cfs_quota_us": "-1\n",
                                "sys/fs/cgroup/cpu,cpuacct/cpu.cfs_period_us": "100000\n"}, None),
        ("0::/\n", {"sys/fs/cgroup/cpu.max": "max 100000\n"}, None),
    ]
    for i, (self_cg, files, quota) in enumerate(cases):
        root = _cgroup_tree(tmp_path / str(i), self_cg, files)
        want = min(aff, quota) if quota else aff
        assert hjd.cpu_share(root) == want, (i, hjd.cpu_share(root), want)
