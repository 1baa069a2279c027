"""The reference's BLS pool metrics, emitted by BlsGpuVerifier.

Names, labels and meaning follow packages/beacon-node/src/metrics/metrics/lodestar.ts:380-495
(`bls.aggregatedPubkeys` and `blsThreadPool.*`) and the update sites in
chain/bls/multithread/index.ts (:148-150, 165-175, 396-404, 433-437, 495-502, 566-567), with
GPUs in place of worker threads (`workerId` = backend index, "busy workers" = busy GPUs).
A plain in-process registry: counters/gauges keyed by (name, labels), histograms
as (count, sum); `collect()` returns a flat dict a Prometheus exporter can serve.
"""
from __future__ import annotations

import threading
from typing import Dict, Tuple

Labels = Tuple[Tuple[str, str], ...]

AGGREGATED_PUBKEYS = "lodestar_bls_aggregated_pubkeys_total"
P = "lodestar_bls_thread_pool_"
JOBS_WORKER_TIME = P + "time_seconds_sum"                      # {workerId}
SUCCESS_JOBS_SETS = P + "success_jobs_signature_sets_count"
ERROR_AGGREGATE_SETS = P + "error_aggregate_signature_sets_count"  # {type}
ERROR_JOBS_SETS = P + "error_jobs_signature_sets_count"
JOB_WAIT_TIME = P + "queue_job_wait_time_seconds"              # histogram
QUEUE_LENGTH = P + "queue_length"                              # gauge
WORKERS_BUSY = P + "workers_busy"                              # gauge
JOB_GROUPS_STARTED = P + "job_groups_started_total"
JOBS_STARTED = P + "jobs_started_total"                        # {type}
SIG_SETS_STARTED = P + "sig_sets_started_total"                # {type}
BATCH_RETRIES = P + "batch_retries_total"
BATCH_SIGS_SUCCESS = P + "batch_sigs_success_total"
SAME_MESSAGE_RETRY_JOBS = P + "same_message_jobs_retries_total"
SAME_MESSAGE_RETRY_SETS = P + "same_message_sets_retries_total"
MAIN_THREAD_TIME = P + "main_thread_time_seconds"              # histogram
TIME_PER_SIG_SET = "lodestar_bls_worker_thread_time_per_sigset_seconds"  # histogram
TOTAL_SIG_SETS = P + "sig_sets_total"
PRIORITIZED_SIG_SETS = P + "prioritized_sig_sets_total"
BATCHABLE_SIG_SETS = P + "batchable_sig_sets_total"
LATENCY_TO_WORKER = P + "latency_to_worker"                    # histogram (dispatch -> GPU submission thread)
LATENCY_FROM_WORKER = P + "latency_from_worker"                # histogram (verdicts ready -> event loop)
SIG_DESERIALIZATION_MAIN_THREAD = P + "signature_deserialization_main_thread_time_seconds"  # GPU decode stage
PUBKEYS_AGGREGATION_MAIN_THREAD = P + "pubkeys_aggregation_main_thread_time_seconds"      # GPU aggregation stage
SINGLE_THREAD_TIME = "lodestar_bls_single_thread_time_seconds"                  # histogram
SINGLE_THREAD_TIME_PER_SIGSET = "lodestar_bls_single_thread_time_per_sigset_seconds"  # histogram


class BlsPoolMetrics:
    def __init__(self):
        self._lock = threading.Lock()
        self._values: Dict[Tuple[str, Labels], float] = {}
        self._hist: Dict[Tuple[str, Labels], Tuple[int, float]] = {}

    @staticmethod
    def _key(name: str, labels: Dict[str, object]) -> Tuple[str, Labels]:
        return name, tuple(sorted((k, str(v)) for k, v in labels.items()))

    def inc(self, name: str, value: float = 1.0, **labels) -> None:
        k = self._key(name, labels)
        with self._lock:
            self._values[k] = self._values.get(k, 0.0) + value

    def set(self, name: str, value: float, **labels) -> None:
        with self._lock:
            self._values[self._key(name, labels)] = float(value)

    def observe(self, name: str, value: float, **labels) -> None:
        k = self._key(name, labels)
        with self._lock:
            c, s = self._hist.get(k, (0, 0.0))
            self._hist[k] = (c + 1, s + float(value))

    def get(self, name: str, **labels) -> float:
        return self._values.get(self._key(name, labels), 0.0)

    def histogram(self, name: str, **labels) -> Tuple[int, float]:
        return self._hist.get(self._key(name, labels), (0, 0.0))

    def collect(self) -> Dict[str, float]:
        """Flat exposition: name{labels} -> value; histograms as name_count / name_sum."""
        out = {}

        def fmt(name, labels, suffix=""):
            lab = ",".join(f'{k}="{v}"' for k, v in labels)
            return f"{name}{suffix}" + (f"{{{lab}}}" if lab else "")
        with self._lock:
            for (name, labels), v in self._values.items():
                out[fmt(name, labels)] = v
            for (name, labels), (c, s) in self._hist.items():
                out[fmt(name, labels, "_count")] = c
                out[fmt(name, labels, "_sum")] = s
        return out
