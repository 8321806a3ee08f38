"""Metric families of the BLS verifier, named as the reference pool's.

Reference: packages/beacon-node/src/metrics/metrics/lodestar.ts:401-504 (``blsThreadPool``) -- the
same family names, label names and histogram buckets, so dashboards built on the worker pool keep
working when GpuBlsVerifier replaces it.  A "worker" here is the device: ``workersBusy`` counts
device passes in flight, the worker time is device wall time per pass.  Families with no pool
counterpart carry ``_gpu_`` in their names.

Every verifier owns its own registry (``prometheus_client.CollectorRegistry``); ``exposition()``
renders it in the Prometheus text format.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Callable, Optional

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

JOB_TYPES = ("default", "sameMessage")  # JobQueueItemType (multithread/jobItem.ts:9)


def observe_many(hist: Histogram, values) -> None:
    """``hist.observe(v)`` for every v of a numpy array, in one bucket count: what observe does per
    value (the first upper bound >= v gets the count, the sum gets v), without a Python-level call
    per job of a device pass."""
    import numpy as np
    v = np.asarray(values, dtype=np.float64)
    if not len(v):
        return
    bounds = np.asarray(hist._upper_bounds, dtype=np.float64)
    counts = np.bincount(np.searchsorted(bounds, v, side="left"), minlength=len(bounds))
    for b, c in zip(hist._buckets, counts):
        if c:
            b.inc(int(c))
    hist._sum.inc(float(v.sum()))


class BlsPoolMetrics:
    """Hot-path counts go through ``add`` (a plain dict, ~0.1 us) and reach the prometheus families
    when they are read (``exposition`` / ``value``), the way the reference refreshes queueLength and
    workersBusy on collect (multithread/index.ts:140-145); ``on_collect`` runs first."""

    def __init__(self):
        self._pending = defaultdict(float)
        self.on_collect: Optional[Callable[[], None]] = None
        r = self.registry = CollectorRegistry(auto_describe=True)
        p = "lodestar_bls_thread_pool_"
        # lodestar.ts:402-405 (workerId label: the device ordinal)
        self.jobs_worker_time = Gauge(p + "time_seconds_sum", "Total time spent verifying signature sets measured on the worker",
                                      ["workerId"], registry=r)
        self.success_jobs_signature_sets_count = Gauge(p + "success_jobs_signature_sets_count", "Count of total verified signature sets",
                                                       registry=r)
        self.error_aggregate_signature_sets_count = Gauge(p + "error_aggregate_signature_sets_count",
                                                          "Count of error when aggregating pubkeys or signatures", ["type"], registry=r)
        self.error_jobs_signature_sets_count = Gauge(p + "error_jobs_signature_sets_count", "Count of total error-ed signature sets",
                                                     registry=r)
        self.job_wait_time = Histogram(p + "queue_job_wait_time_seconds", "Time from job added to the queue to starting the job in seconds",
                                       buckets=sorted([0.01, 0.02, 0.5, 0.1, 0.3, 1]), registry=r)  # prom-client sorts the reference's list
        self.queue_length = Gauge(p + "queue_length", "Count of total block processor queue length", registry=r)
        self.workers_busy = Gauge(p + "workers_busy", "Count of current busy workers", registry=r)
        self.total_jobs_groups_started = Gauge(p + "job_groups_started_total",
                                               "Count of total jobs groups started in bls thread pool, job groups include +1 jobs", registry=r)
        self.total_jobs_started = Gauge(p + "jobs_started_total",
                                        "Count of total jobs started in bls thread pool, jobs include +1 signature sets", ["type"], registry=r)
        self.total_sig_sets_started = Gauge(p + "sig_sets_started_total",
                                            "Count of total signature sets started in bls thread pool, sig sets include 1 pk, msg, sig",
                                            ["type"], registry=r)
        self.batch_retries = Gauge(p + "batch_retries_total", "Count of total batches that failed and had to be verified again.", registry=r)
        self.batch_sigs_success = Gauge(p + "batch_sigs_success_total", "Count of total batches that failed and had to be verified again.",
                                        registry=r)
        self.same_message_retry_jobs = Gauge(p + "same_message_jobs_retries_total",
                                             "Count of total same message jobs that failed and had to be verified again.", registry=r)
        self.same_message_retry_sets = Gauge(p + "same_message_sets_retries_total",
                                             "Count of total same message sets that failed and had to be verified again.", registry=r)
        self.latency_to_worker = Histogram(p + "latency_to_worker", "Time from sending the job to the worker and the worker receiving it",
                                           buckets=[0.001, 0.003, 0.01, 0.03, 0.1], registry=r)
        self.latency_from_worker = Histogram(p + "latency_from_worker",
                                             "Time from the worker sending the result and the main thread receiving it",
                                             buckets=[0.001, 0.003, 0.01, 0.03, 0.1], registry=r)
        self.main_thread_duration_in_thread_pool = Histogram(p + "main_thread_time_seconds",
                                                             "Time to verify signatures in main thread with thread pool mode", buckets=[0],
                                                             registry=r)
        self.time_per_sig_set = Histogram("lodestar_bls_worker_thread_time_per_sigset_seconds",
                                          "Time to verify each sigset with worker thread mode",
                                          buckets=[0.5e-3, 0.75e-3, 1e-3, 1.5e-3, 2e-3, 5e-3], registry=r)
        self.total_sig_sets = Gauge(p + "sig_sets_total", "Count of total signature sets", registry=r)
        self.prioritized_sig_sets = Gauge(p + "prioritized_sig_sets_total", "Count of total prioritized signature sets", registry=r)
        self.batchable_sig_sets = Gauge(p + "batchable_sig_sets_total", "Count of total batchable signature sets", registry=r)
        self.aggregate_with_randomness_main_thread_duration = Histogram(
            p + "aggregate_with_randomness_main_thread_time_seconds", "Total time performing aggregateWithRandomness on main thread",
            buckets=[0.001, 0.005, 0.01, 0.1], registry=r)
        self.pubkeys_aggregation_main_thread_duration = Histogram(
            p + "pubkeys_aggregation_main_thread_time_seconds", "Total time spent aggregating pubkeys on main thread",
            buckets=[0.001, 0.005, 0.01, 0.1], registry=r)
        # device-only families
        self.gpu_device_passes = Counter(p + "gpu_device_passes", "Device passes (one or more jobs verified together)", registry=r)
        self.gpu_pass_sets = Histogram(p + "gpu_pass_sig_sets", "Signature sets per device pass",
                                       buckets=[1, 16, 128, 1024, 8192, 65536, 262144], registry=r)
        self.gpu_pass_time = Histogram(p + "gpu_pass_time_seconds", "Device pass wall time, submit to results",
                                       buckets=[0.005, 0.01, 0.02, 0.05, 0.1, 0.3, 1], registry=r)

    def add(self, family: str, v: float = 1.0, label: Optional[str] = None):
        self._pending[(family, label)] += v

    def flush(self):
        if self.on_collect is not None:
            self.on_collect()
        pend, self._pending = self._pending, defaultdict(float)
        for (family, label), v in pend.items():
            f = getattr(self, family)
            (f.labels(label) if label is not None else f).inc(v)

    def exposition(self) -> bytes:
        self.flush()
        return generate_latest(self.registry)

    def value(self, name: str, labels: dict | None = None) -> float:
        self.flush()
        v = self.registry.get_sample_value(name, labels or {})
        return 0.0 if v is None else float(v)
