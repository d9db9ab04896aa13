// sprof.c -- development tool: a minimal sampling CPU profiler for the host driver
// (no perf in the dev container).  LD_PRELOAD it; every SPROF_HZ of process CPU time
// (ITIMER_PROF, default 997 Hz) the running thread records its PC and a few return
// addresses; at exit the samples are symbolised with dladdr and the flat profile
// (self) and the inclusive counts of the first frames are written to $SPROF_OUT
// (default sprof.txt).  Build the profiled binary with -rdynamic so its own symbols
// resolve.  SPROF_WAIT=1 samples only after the program raises SIGUSR2
// (tests/cpp/test_e2e_oracle --host-timing does before its timed replay pass).
// SPROF_RAW=file also writes every sample's frames as module:offset, for
// tools/sprof_report.py (addr2line: static functions and inlined frames resolve too).
//   gcc -O2 -shared -fPIC -o /tmp/sprof.so tools/sprof.c -ldl
//   SPROF_OUT=/tmp/p.txt LD_PRELOAD=/tmp/sprof.so ./binary ...
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <ucontext.h>

#define MAXS (1 << 21)
#define DEPTH 6
static void* g_pc[MAXS][DEPTH];
static atomic_int g_n;
static volatile sig_atomic_t g_on = 1;          // SPROF_WAIT=1: off until the program raises SIGUSR2
static void on_usr2(int sig) { (void)sig; g_on = !g_on; }   // each SIGUSR2 toggles sampling

static void on_prof(int sig, siginfo_t* si, void* uc_) {
	(void)sig; (void)si;
	if(!g_on) return;
	const int k = atomic_fetch_add(&g_n, 1);
	if(k >= MAXS) return;
	ucontext_t* uc = (ucontext_t*)uc_;
	void* bt[DEPTH + 2];
	const int n = backtrace(bt, DEPTH + 2);
	g_pc[k][0] = (void*)uc->uc_mcontext.gregs[REG_RIP];
	// bt[0] is this handler, bt[1] the signal trampoline; then the interrupted frames'
	// callers (bt[2] is usually the interrupted function itself)
	for(int d = 1; d < DEPTH; d++) g_pc[k][d] = (d + 2 < n) ? bt[d + 2] : NULL;
}

static const char* sym(void* pc, char* buf, size_t nb) {
	Dl_info di;
	if(pc && dladdr(pc, &di) && di.dli_sname) return di.dli_sname;
	if(pc && dladdr(pc, &di) && di.dli_fname) {
		const char* b = strrchr(di.dli_fname, '/');
		snprintf(buf, nb, "[%s]", b ? b + 1 : di.dli_fname);
		return buf;
	}
	return "?";
}

typedef struct { const char* name; long self, incl; } Ent;
static Ent* g_ent; static int g_nent;
static Ent* find(const char* name) {
	for(int i = 0; i < g_nent; i++) if(!strcmp(g_ent[i].name, name)) return &g_ent[i];
	g_ent[g_nent].name = strdup(name);
	g_ent[g_nent].self = g_ent[g_nent].incl = 0;
	return &g_ent[g_nent++];
}
static int by_self(const void* a, const void* b) { return (int)(((const Ent*)b)->self - ((const Ent*)a)->self); }

__attribute__((constructor)) static void sprof_init(void) {
	void* warm[4];
	backtrace(warm, 4);                           // loads libgcc_s before the first signal
	struct sigaction sa;
	memset(&sa, 0, sizeof sa);
	sa.sa_sigaction = on_prof;
	sa.sa_flags = SA_SIGINFO | SA_RESTART;
	sigaction(SIGPROF, &sa, NULL);
	if(getenv("SPROF_WAIT")) { g_on = 0; signal(SIGUSR2, on_usr2); }
	const char* hz = getenv("SPROF_HZ");
	const long us = 1000000 / (hz ? atol(hz) : 997);
	struct itimerval it = {{0, us}, {0, us}};
	setitimer(ITIMER_PROF, &it, NULL);
}

__attribute__((destructor)) static void sprof_fini(void) {
	struct itimerval it = {{0, 0}, {0, 0}};
	setitimer(ITIMER_PROF, &it, NULL);
	int n = atomic_load(&g_n);
	if(n > MAXS) n = MAXS;
	g_ent = calloc(65536, sizeof(Ent));
	char buf[256];
	for(int k = 0; k < n; k++) {
		find(sym(g_pc[k][0], buf, sizeof buf))->self++;
		const char* seen[DEPTH];
		int ns = 0;
		for(int d = 0; d < DEPTH && g_nent < 65000; d++) {
			if(!g_pc[k][d]) break;
			const char* s = find(sym(g_pc[k][d], buf, sizeof buf))->name;
			int dup = 0;
			for(int j = 0; j < ns; j++) if(seen[j] == s) dup = 1;
			if(!dup) { seen[ns++] = s; find(s)->incl++; }
		}
	}
	const char* raw = getenv("SPROF_RAW");         // per sample: module:offset of each frame
	if(raw) {
		FILE* fr = fopen(raw, "w");
		for(int k = 0; fr && k < n; k++) {
			for(int d = 0; d < DEPTH && g_pc[k][d]; d++) {
				Dl_info di;
				if(dladdr(g_pc[k][d], &di) && di.dli_fname)
					fprintf(fr, "%s%s:%lx", d ? " " : "", di.dli_fname,
					        (unsigned long)((char*)g_pc[k][d] - (char*)di.dli_fbase) - (d ? 1 : 0));
				else fprintf(fr, "%s?", d ? " " : "");
			}
			fputc('\n', fr);
		}
		if(fr) fclose(fr);
	}
	qsort(g_ent, g_nent, sizeof(Ent), by_self);
	const char* out = getenv("SPROF_OUT");
	FILE* f = fopen(out ? out : "sprof.txt", "w");
	if(!f) return;
	fprintf(f, "# %d samples; self%% incl%%(first %d frames) symbol\n", n, DEPTH);
	for(int i = 0; i < g_nent; i++)
		if(g_ent[i].self * 1000 >= n || g_ent[i].incl * 200 >= n)
			fprintf(f, "%6.2f %6.2f %s\n", 100.0 * g_ent[i].self / n, 100.0 * g_ent[i].incl / n, g_ent[i].name);
	fclose(f);
}
