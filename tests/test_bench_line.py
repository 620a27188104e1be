"""bench.py's stdout line: the driver keeps only the last
~2 KB of stdout, so the line is compact and ends with a `summary` holding
every leg's headline number -- configs[2] and configs[3] with value, ms and
roofline fraction, configs[1], both config-5 stream legs and the host-Huffman
one, and the CPU legs -- while the full result goes to a detail file.  Built
here from a committed full result of round 4 (profiles/r04m_bench.json), no
GPU needed."""
import importlib.util
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _full():
    res = json.load(open(os.path.join(REPO, "profiles", "r04m_bench.json")))
    res["config5_stream_host"] = {
        "value": 5900.0, "timed_frame_ids": 10240, "output_checked_vs_oracle": True,
        "pipeline": {"host_huffman_Mpx_per_core_s": 380.1, "host_threads": 16, "h2d_GBps": 2.1,
                     "kernel_busy_frac": 0.0213, "h2d_busy_frac": 0.05, "kernel_only_Mpx_s": 318000.5,
                     "pcie_ceiling_Mpx_s": 18500.2}}
    return res


def test_compact_line_fits_the_driver_tail():
    b = _bench()
    line = json.dumps(b.compact_line(_full(), "gpurun_out/bench_detail.json"))
    assert len(line) < 1900, len(line)
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert list(d)[-1] == "summary"          # the tail always holds it
    s = d["summary"]
    for leg in ("4k420", "4k444"):
        assert {"Mpx_s", "ms", "frac", "box_frac", "ok"} <= set(s[leg]), s[leg]
    assert s["4k444"]["frac"] == _full()["config4_444"]["roofline"]["frac"]
    assert s["c5_host_huffman"]["kernel_busy"] == 0.0213
    assert s["c5_gpu_huffman"]["h2d_frac"] and s["c5_d2h"]["d2h_frac"]
    assert d["output_checked_vs_oracle"] is True


def test_compact_line_reports_a_failed_leg():
    b = _bench()
    res = _full()
    res["config4_444"]["output_checked_vs_oracle"] = False
    res["config5_stream_d2h"] = {"error": "rc 1", "stderr_tail": "x" * 400}
    d = b.compact_line(res, "x.json")
    assert d["output_checked_vs_oracle"] is False
    assert d["summary"]["c5_d2h"] == {"error": "rc 1"}


def test_emit_writes_detail(tmp_path, capsys):
    b = _bench()
    res = _full()
    path = str(tmp_path / "sub" / "detail.json")
    b.emit(res, path)
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1 and json.loads(out[0])["detail"] == path
    assert json.load(open(path))["config4_444"]["value"] == res["config4_444"]["value"]
