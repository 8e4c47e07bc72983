/*
 * Synthetic corpus generator (benchmark / test utility, not part of the
 * evaluation boundary). Produces NDJSON resources shaped like SURVEY.md §8(d):
 *   C2: Pods with 1-4 containers (p=.7/.2/.07/.03), 0-1 initContainers (p=.8/.2),
 *       ~60% restricted-compliant (docs/perf-testing/main.go:201-246 template),
 *       ~40% with 1-3 violations drawn uniformly from the 17 PSA checks, fields
 *       present or absent at p=0.5, namespaces ns-0000..ns-0999, images from
 *       50 names x {latest, semver}.
 * Deterministic in (seed, first_index): row i of a corpus depends only on
 * (seed, first_index + i), so shards of one logical corpus can be generated
 * independently per rank.
 */
#ifndef KPE_SYNTH_H_
#define KPE_SYNTH_H_
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum kpe_synth_mix {
  KPE_SYNTH_PODS = 0,   /* C2: Pods only                                      */
  KPE_SYNTH_MIXED = 1,  /* Pods, Deployments, DaemonSets, Jobs, CronJobs, Services, ConfigMaps */
  KPE_SYNTH_EDGE = 2,   /* MIXED + edge cases: nulls, windows pods, type errors, odd values */
  KPE_SYNTH_SELECTORS = 3, /* C4: Deployments + Services, 8 labels from a 64-key vocabulary,
                             namespaces ns-00000..ns-09999 */
  KPE_SYNTH_FANOUT = 4,   /* C5: Pods (85%) and Deployments with 1-64 containers (truncated
                             geometric, mean ~6) + 0-3 initContainers; images with / without
                             tags, digests, registries; resources.requests/limits present,
                             partial, empty or absent; ports with / without hostPort */
  KPE_SYNTH_C3 = 5        /* C3: Pod 40%, Deployment 20%, Service 15%, ConfigMap 15%,
                             Job / CronJob / StatefulSet 10%; names app-<word>-<c>, web-*,
                             *-canary, *-db-*; namespaces team-<k>[-prod|-dev], *-prod,
                             kube-system, default */
};

/* Generate n resources as NDJSON into a malloc'd buffer (*out, *len). Free with kpe_synth_free. */
int kpe_synth_resources(uint64_t seed, int64_t first_index, int64_t n, int mix, char** out, size_t* len);
void kpe_synth_free(char* p);
/* Namespace label table {"ns-…": {"k": "v"}} for namespaces 0..n-1 of the given mix
 * (ns-%04d, or ns-%05d for KPE_SYNTH_SELECTORS). Free with kpe_synth_free. */
int kpe_synth_ns_labels(uint64_t seed, int64_t n_namespaces, int mix, char** out, size_t* len);

#ifdef __cplusplus
}
#endif
#endif
