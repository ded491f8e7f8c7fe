"""The measurement tooling on CPU: tools/pmc_traffic.py folds rocprofv3 counter CSVs into the
per-launch table bench.py reads (roofline.traffic and the counter fractions), keyed the way the
bench names its workloads, with the build id of the library the passes ran."""
import csv
import json
import os
import subprocess
import sys

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, 'tools'))


def _counters(path, kernel, per_dispatch, other='void wrnn::k_gemm<4, 0, 16>(int)'):
    """A run_counter_collection.csv of 2 dispatches of `kernel` (each counter split over two
    dimension rows, as rocprofv3 reports per-XCD instances) and one dispatch of another kernel."""
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, 'w', newline='') as f:
        w = csv.DictWriter(f, fieldnames=['Dispatch_Id', 'Kernel_Name', 'Counter_Name', 'Counter_Value'])
        w.writeheader()
        for d in (1, 2):
            for name, v in per_dispatch.items():
                for half in (0.25, 0.75):
                    w.writerow({'Dispatch_Id': d, 'Kernel_Name': kernel, 'Counter_Name': name,
                                'Counter_Value': v * d * half})
        for name in per_dispatch:
            w.writerow({'Dispatch_Id': 3, 'Kernel_Name': other, 'Counter_Name': name, 'Counter_Value': 1e9})


def test_pmc_fold_is_per_launch_of_the_named_kernel(tmp_path):
    import pmc_traffic
    src = tmp_path / 'pmc'
    rr_kernel = 'void wrnn::k_persist_wide_rr<false>(wrnn::PersistRRArgs)'
    _counters(str(src / 'rr_fetch' / 'run_counter_collection.csv'), rr_kernel, {'FETCH_SIZE': 1000.0})
    _counters(str(src / 'rr_write' / 'run_counter_collection.csv'), rr_kernel, {'WRITE_SIZE': 300.0})
    sq = {'SQ_WAVE_CYCLES': 1e6, 'SQ_BUSY_CYCLES': 5e5, 'SQ_WAIT_ANY': 4e5, 'SQ_WAIT_INST_ANY': 1e5,
          'SQ_ACTIVE_INST_ANY': 2e5, 'SQ_VALU_MFMA_BUSY_CYCLES': 1024 * 1000.0,
          'SQ_LDS_BANK_CONFLICT': 10.0, 'SQ_LDS_IDX_ACTIVE': 100.0, 'GRBM_GUI_ACTIVE': 8 * 4000.0}
    _counters(str(src / 'rr_sq' / 'run_counter_collection.csv'), rr_kernel, sq)
    (src / 'lib_build').write_text('0123456789abcdef\n')
    table = tmp_path / 'table.json'
    subprocess.run([sys.executable, os.path.join(REPO, 'tools', 'pmc_traffic.py'), str(src),
                    str(tmp_path / 'round'), str(table)], check=True, capture_output=True)
    t = json.load(open(table))
    key = 'k_persist_wide_rr|' + pmc_traffic.WORKLOADS['rr'][1]
    e = t[key]
    # dispatches carry 1x and 2x the counters: the per-launch mean is 1.5x, the other kernel ignored
    assert e['launches'] == 2 and e['kernel'] == rr_kernel
    assert e['fetch_size_kib'] == 1500.0 and e['write_size_kib'] == 450.0
    assert e['traffic_bytes'] == (2 * 1500.0 + 450.0) * 1024  # FETCH_SIZE doubled (gfx950)
    assert e['lib_build'] == '0123456789abcdef'
    assert abs(e['mfma_busy_frac'] - 1.5 * 1024 * 1000.0 / (1024 * 1.5 * 4000.0)) < 1e-12
    assert abs(e['wait_frac'] - 0.4) < 1e-12 and abs(e['lds_conflict_frac'] - 0.1) < 1e-12
    assert os.path.exists(tmp_path / 'round' / 'pmc' / 'rr_fetch.csv')


def test_workload_keys_are_the_bench_strings():
    import bench
    import pmc_traffic
    cases = {'c2': ('fatchord-wavernn', 'RAW 9-bit mu-law', 1, 11000, 550),
             'c4': ('fatchord-wavernn', 'RAW 9-bit mu-law', 8, 11000, 550),
             'c3': ('fatchord-wavernn', 'MOL', 1, 11000, 550),
             'rr': ('runtimeracer-wavernn', 'RAW 10-bit mu-law', 8, 6000, 1000)}
    for k, (model, wname, u, tgt, ovl) in cases.items():
        assert pmc_traffic.WORKLOADS[k][1] == bench.workload_of(u, 1000, model, wname, tgt, ovl), k


def test_bench_reads_the_table_it_is_pointed_at(tmp_path, monkeypatch):
    import bench
    path = tmp_path / 't.json'
    path.write_text(json.dumps({'k_persist|w': {'traffic_bytes': 5.0, 'lib_build': 'x'}}))
    monkeypatch.setenv('WRNN_PMC_TRAFFIC', str(path))
    assert bench._pmc_traffic('k_persist', 'w')['traffic_bytes'] == 5.0
    assert bench._pmc_traffic('k_persist', 'other') is None
    monkeypatch.setenv('WRNN_PMC_TRAFFIC', str(tmp_path / 'missing.json'))
    assert bench._pmc_traffic('k_persist', 'w') is None
