"""bench.py's launcher: `python bench.py --gpus N` outside torch.distributed.run
starts its own N ranks as a child process, before anything touches torch or the GPU, relays rank
0's line and fails when a rank fails; under torch.distributed.run it is one rank."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_needs_launch():
    assert bench.needs_launch(2, {})
    assert bench.needs_launch(8, {'RANK': '0'})
    assert not bench.needs_launch(1, {})
    assert not bench.needs_launch(2, {'WORLD_SIZE': '2'})      # already a rank


def test_launcher_cmd():
    cmd = bench.launcher_cmd(4, ['--gpus', '4', '--steps', '3'], 29555)
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert cmd[cmd.index('--nproc-per-node') + 1] == '4'
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[cmd.index('--master-port') + 1] == '29555'
    assert cmd[-4:] == ['--gpus', '4', '--steps', '3']
    assert cmd[-5] == os.path.abspath(bench.__file__)


def test_defaults_one_workload_every_n():
    """The default workload is the same at every N (a 1 -> 8 series is one curve)."""
    assert bench.parse([]).workload == 'c3'
    assert bench.parse(['--gpus', '8']).workload == 'c3'
    assert bench.WORKLOADS['c3']['scaling'] == 'strong' and bench.WORKLOADS['c5']['scaling'] == 'weak'


def test_import_does_not_load_torch():
    """The parent must not touch torch / HIP before it starts the ranks."""
    code = 'import sys; sys.path.insert(0, %r); import bench; assert "torch" not in sys.modules' % ROOT
    subprocess.run([sys.executable, '-c', code], check=True, timeout=60)


def _fake_rank_script(tmp_path, fail_rank=None):
    p = tmp_path / 'fake_rank.py'
    p.write_text(
        'import os, sys, json\n'
        'r = int(os.environ["RANK"]); w = int(os.environ["WORLD_SIZE"])\n'
        'assert "--gpus" in sys.argv\n'
        'if r == %r: sys.exit(3)\n'
        'if r == 0: print(json.dumps({"n_gpus": w, "argv": sys.argv[1:]}), flush=True)\n' % fail_rank)
    return str(p)


def _run_launcher(script, n):
    code = ('import sys; sys.path.insert(0, %r); import bench; '
            'bench.launcher_cmd.__defaults__ = (%r,); '
            'sys.exit(bench.self_launch(%d, ["--gpus", "%d", "--steps", "2"]))' % (ROOT, script, n, n))
    return subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize('n', [2, 3])
def test_self_launch_relays_rank0_line(tmp_path, n):
    import json
    r = _run_launcher(_fake_rank_script(tmp_path), n)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d['n_gpus'] == n and d['argv'] == ['--gpus', str(n), '--steps', '2']


def test_self_launch_fails_when_a_rank_fails(tmp_path):
    r = _run_launcher(_fake_rank_script(tmp_path, fail_rank=1), 2)
    assert r.returncode != 0


def test_traffic_file_provenance(tmp_path):
    """roofline.traffic comes only from a traffic file stamped with the benched library's source
    hash (tools/prof_summary.py --bench-json); unstamped or stale files give None."""
    import json
    p = tmp_path / 't.json'
    body = {'k_pass2<true>': {'traffic': 34940478334}, 'k_spec<false, 1, 0>': {'traffic': 18212456067}}
    p.write_text(json.dumps(body))
    assert bench.load_traffic(str(p), 'k_pass2', 'abc') == (None, None)          # unstamped
    p.write_text(json.dumps(dict({'_meta': {'lib_src': 'old'}}, **body)))
    assert bench.load_traffic(str(p), 'k_pass2', 'abc') == (None, 'old')         # another build
    p.write_text(json.dumps(dict({'_meta': {'lib_src': 'abc'}}, **body)))
    assert bench.load_traffic(str(p), 'k_pass2', 'abc') == (34940478334, 'abc')
    assert bench.load_traffic(str(p), 'k_spec', 'abc') == (18212456067, 'abc')
    assert bench.load_traffic(str(tmp_path / 'none.json'), 'k_pass2', 'abc') == (None, None)
