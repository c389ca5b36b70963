// vafc_affinity.h -- CPU placement of the host reader threads (vc_count_file).
//
// The counting pass of a FASTQ file is bound by its host stages (parse,
// inflate): reader threads parse the page-cached text
// into pinned slots that the GPU then copies.  vc_count_file binds those
// threads to the CPUs of the NUMA node the counter's GPU hangs off (sysfs,
// from the device's PCI bus id), intersected with the process's own affinity
// mask: the slots are DMA'd from that node's memory, and a thread that the
// scheduler moves across sockets mid-pass was the spread's suspected cause.
// The calling thread publishes the set in a thread-local; every thread the
// readers spawn (parse workers, inflate workers, the gzip pump) copies it at
// creation and binds itself.  VAFC_NUMA=0 turns the binding off.
#ifndef VAFC_AFFINITY_H
#define VAFC_AFFINITY_H
#include <pthread.h>
#include <sched.h>

struct VcCpuSet {
	cpu_set_t set;
	bool on = false;
};

inline thread_local VcCpuSet vc_tl_cpus;

// The current thread's published set (what new reader threads bind to).
inline VcCpuSet vc_affinity_get() { return vc_tl_cpus; }

// Bind the calling thread to s (no-op when s is off).
inline void vc_affinity_bind(const VcCpuSet &s)
{
	if (s.on) (void)pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), &s.set);
}

// Publishes a set for the threads this thread spawns while in scope.
struct VcAffinityScope {
	VcCpuSet saved;
	explicit VcAffinityScope(const VcCpuSet &s) : saved(vc_tl_cpus) { vc_tl_cpus = s; }
	~VcAffinityScope() { vc_tl_cpus = saved; }
};

#endif
