#!/usr/bin/env python3
"""Benchmark entry point of the reference (scripts/benchmark_sequential.py),
now driving the MI355X builder through a thin ctypes shim over the C ABI.

Kept from the reference (a-rtemis99/hpc_suffix_array):
  * main() / run_benchmark(input_file) / parse_output(output) / format_time
  * the input file list (:155-166) and "NON TROVATO" for missing files
  * the 16-column CSV at results/benchmarks/sequential_results.csv (:192-223)
  * the stdout text contract parse_output reads (:13-72)
Changed: run_benchmark no longer spawns ./bin/main_sequential (:76-85); it
calls create/build/lcp/lrs/is_valid of libsa_hip.so in-process (the same
six symbols of suffix_array.h) and renders the same text the CLI prints, so
parse_output is unchanged.  `--cli` runs bin/main_sequential instead (the
C driver with the reference's stdout contract, tools/sa_main.c).
Input files: scripts/generate_large_datasets.py (seeded splitmix64).
"""
import argparse
import os
import re
import subprocess
import sys
import time
from datetime import datetime

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEQUENTIAL_FILES = [
    "test_data/banana.txt",
    "test_data/mississippi.txt",
    "test_data/abcabcabc.txt",
    "test_data/aaaa.txt",
    "test_data/ababab.txt",
    "test_data/large/random_1MB.txt",
    "test_data/large/random_50MB.txt",
    "test_data/large/random_100MB.txt",
    "test_data/large/random_200MB.txt",
    "test_data/large/random_500MB.txt",
]

CSV_COLUMNS = ["file", "size_bytes", "size_mb", "backend", "time_seconds", "throughput_mb_s",
               "throughput_chars_per_second", "lrs_length", "lrs_string", "suffix_array_length",
               "execution_details", "total_time", "sa_time", "lcp_time", "success", "timestamp"]


def parse_output(output):
    """Same keys and regular expressions as the reference (:13-72)."""
    result = {'lrs_length': 0, 'lrs_string': 'N/A', 'suffix_array_length': 0, 'execution_details': 'N/A',
              'total_time': 0.0, 'sa_time': 0.0, 'lcp_time': 0.0}
    for line in output.split('\n'):
        if 'Longest repeated substring:' in line and 'length:' in line:
            m = re.search(r'length:\s*(\d+)', line)
            if m:
                result['lrs_length'] = int(m.group(1))
            m = re.search(r"substring:\s*'([^']*)'", line) or re.search(r'substring:\s*"([^"]*)"', line)
            if m:
                result['lrs_string'] = m.group(1)
        if 'Actual string length:' in line:
            m = re.search(r'Actual string length:\s*(\d+)', line)
            if m:
                result['suffix_array_length'] = int(m.group(1))
        if 'Total execution time:' in line:
            m = re.search(r'Total execution time:\s*([\d.]+)', line)
            if m:
                result['total_time'] = float(m.group(1))
                result['execution_details'] = line.strip()
        for key, name in (('TOTAL_TIME:', 'total_time'), ('SA_TIME:', 'sa_time'), ('LCP_TIME:', 'lcp_time')):
            if key in line:
                m = re.search(key + r'([\d.]+)', line)
                if m:
                    result[name] = float(m.group(1))
    return result


def shim_run(input_file):
    """The CLI's work and stdout text, in-process through the C ABI
    (main_sequential.c:60-154 semantics: SA_TIME = create + build,
    LCP_TIME = LCP + LRS, validation untimed)."""
    from hpc_suffix_array_amd import SuffixArray
    with open(input_file, "rb") as f:
        data = f.read()
    n = len(data)
    out = [f"Reading from file: {input_file}", f"File read successfully: {input_file}",
           f"Actual string length: {n}", ""]
    t0 = time.time()
    s = SuffixArray(data)
    s.build()
    t_mid = time.time()
    s.build_lcp()
    lrs = s.longest_repeated_substring()
    t_end = time.time()
    valid = s.is_valid()
    s.close()
    out.append("=== RESULTS ===")
    out.append(f"Valid suffix array: {'YES' if valid else 'NO'}")
    if lrs:
        out.append(f"Longest repeated substring: '{lrs.decode('latin-1')}' (length: {len(lrs)})")
    else:
        out.append("No repeated substring found")
    out.append(f"Suffix array construction time: {t_mid - t0:.6f} seconds")
    out.append(f"LCP construction + LRS search time: {t_end - t_mid:.6f} seconds")
    out.append(f"Total execution time: {t_end - t0:.6f} seconds")
    out += ["", "===STRUCTURED_RESULTS===", "IMPLEMENTATION:hip_gpu", f"FILENAME:{input_file}",
            f"FILE_SIZE:{n}", f"TOTAL_TIME:{t_end - t0:.6f}", f"SA_TIME:{t_mid - t0:.6f}",
            f"LCP_TIME:{t_end - t_mid:.6f}", "PROCESSES:1", "===END_RESULTS===", ""]
    return "\n".join(out)


def run_benchmark(input_file, use_cli=False):
    """Runs one file; returns the reference's result dict (:74-130)."""
    start = time.time()
    try:
        if use_cli:
            r = subprocess.run([os.path.join(ROOT, "bin", "main_sequential"), input_file], capture_output=True,
                               text=True, timeout=7200)
            ok, stdout, err = r.returncode == 0, r.stdout, r.stderr
        else:
            stdout, ok, err = shim_run(input_file), True, ""
        elapsed = time.time() - start
        p = parse_output(stdout)
        return dict(success=ok, time=elapsed, output=stdout, error=err, **p)
    except subprocess.TimeoutExpired:
        return dict(success=False, time=7200, error='TIMEOUT', lrs_length=0, lrs_string='TIMEOUT',
                    suffix_array_length=0, execution_details='TIMEOUT', total_time=0.0, sa_time=0.0,
                    lcp_time=0.0)
    except Exception as e:  # noqa: BLE001 -- reported per file, like the reference
        return dict(success=False, time=0, error=str(e), lrs_length=0, lrs_string='ERROR',
                    suffix_array_length=0, execution_details='ERROR', total_time=0.0, sa_time=0.0,
                    lcp_time=0.0)


def format_time(seconds):
    if seconds < 0.001:
        return f"{seconds * 1000:.2f}ms"
    if seconds < 1:
        return f"{seconds * 1000:.0f}ms"
    if seconds < 60:
        return f"{seconds:.2f}s"
    if seconds < 3600:
        return f"{seconds / 60:.1f}m"
    return f"{seconds / 3600:.1f}h"


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--cli", action="store_true", help="run bin/main_sequential instead of the ctypes shim")
    ap.add_argument("--files", nargs="*", default=SEQUENTIAL_FILES)
    ap.add_argument("--out", default="results/benchmarks/sequential_results.csv")
    a = ap.parse_args(argv)
    import pandas as pd
    print("BENCHMARK SEQUENZIALE - Suffix Array (MI355X / libsa_hip)")
    print("=" * 60)
    print(f"Avviato: {datetime.now().strftime('%Y-%m-%d %H:%M:%S')}\n")
    rows, ok_count = [], 0
    for f in a.files:
        if not os.path.exists(f):
            print(f"{os.path.basename(f):25} - NON TROVATO")
            continue
        size = os.path.getsize(f)
        mb = size / (1024 * 1024)
        print(f"{os.path.basename(f):25} ({mb:6.1f} MB)...", end=" ", flush=True)
        r = run_benchmark(f, use_cli=a.cli)
        if not r['success']:
            print("FAILED")
            if r['error']:
                print(f"      Error: {r['error'][:100]}")
            continue
        ok_count += 1
        print(f"{format_time(r['time']):>8} - LRS: {r['lrs_length']:3} chars ('{r['lrs_string'][:20]}')")
        rows.append({'file': os.path.basename(f), 'size_bytes': size, 'size_mb': mb, 'backend': 'hip_gpu',
                     'time_seconds': r['time'], 'throughput_mb_s': mb / r['time'] if r['time'] > 0 else 0,
                     'throughput_chars_per_second': size / r['time'] if r['time'] > 0 else 0,
                     'lrs_length': r['lrs_length'], 'lrs_string': r['lrs_string'],
                     'suffix_array_length': r['suffix_array_length'],
                     'execution_details': r['execution_details'], 'total_time': r['total_time'],
                     'sa_time': r['sa_time'], 'lcp_time': r['lcp_time'], 'success': True,
                     'timestamp': datetime.now()})
    if not rows:
        print("\nNessun test completato con successo!")
        return 1
    df = pd.DataFrame(rows, columns=CSV_COLUMNS)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    df.to_csv(a.out, index=False)
    print("\n" + "=" * 60)
    print(f"Risultati salvati: {a.out}")
    print(f"Test completati: {ok_count}/{len(a.files)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
