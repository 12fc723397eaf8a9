"""One-screen digest of a kgwe.bench.sched_latency JSON result."""
import json
import sys

d = json.load(open(sys.argv[1]))
keys = ("nodes", "arrival_rate_per_s", "bound", "sched_p50_ms", "sched_p99_ms", "p99_ms", "queued_pods",
        "preemptions", "preemption_rate_pct", "preemptions_deferred_wait", "preemptions_rate_limited",
        "non_preemptible_evicted", "throughput_pods_per_s")
print({k: d.get(k) for k in keys})
print("  verbs p50/p99 ms:", {k: (v.get("p50_ms"), v.get("p99_ms"))
                              for k, v in (d.get("extender_phases_ms") or {}).items()})
print("  first cycle p50/p99 ms:", {k: (v.get("p50"), v.get("p99"))
                                    for k, v in (d.get("first_cycle_breakdown_ms") or {}).items()})
