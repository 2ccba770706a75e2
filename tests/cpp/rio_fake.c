/* rio_fake.c — link-time fake of RIORegisterBuffer / RIODeregisterBuffer for the pattern mirror's
 * registered-IO tests (the reference's MSTest projects replace ctsConfig and its rioFunctions by
 * fakes the same way). Built by tests/conftest.py into a temporary .so and installed with
 * cts_rio_functions_set (include/cts_pattern.h).
 *
 * Every registration gets a fresh id (never RIO_INVALID_BUFFERID) and is remembered with its
 * (buffer, length) so a test can check that a task's id names exactly the memory the task points
 * at; deregistering an id that is not live counts as an error. rio_fake_reset(k) makes the
 * (k+1)-th registration from then on fail, as RIORegisterBuffer does when the kernel refuses.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

#define RIO_INVALID 0xFFFFFFFFull

typedef struct {
    uint64_t ptr;
    uint32_t len;
    uint32_t live;
} entry;

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static entry* g_tab = NULL;     /* id i+1 lives at g_tab[i] */
static uint64_t g_n = 0, g_cap = 0;
static uint64_t g_live = 0, g_errors = 0;
static uint64_t g_fail_after = UINT64_MAX;

uint64_t rio_fake_register(void* ctx, char* buffer, uint32_t length)
{
    (void)ctx;
    uint64_t id = RIO_INVALID;
    pthread_mutex_lock(&g_mu);
    if (g_fail_after == 0) goto out;
    if (g_fail_after != UINT64_MAX) --g_fail_after;
    if (buffer == NULL || length == 0) {
        ++g_errors;
        goto out;
    }
    if (g_n == g_cap) {
        const uint64_t cap = g_cap ? 2 * g_cap : 4096;
        entry* t = (entry*)realloc(g_tab, cap * sizeof(entry));
        if (t == NULL) goto out;
        g_tab = t;
        g_cap = cap;
    }
    g_tab[g_n].ptr = (uint64_t)(uintptr_t)buffer;
    g_tab[g_n].len = length;
    g_tab[g_n].live = 1;
    id = ++g_n;
    ++g_live;
out:
    pthread_mutex_unlock(&g_mu);
    return id;
}

void rio_fake_deregister(void* ctx, uint64_t id)
{
    (void)ctx;
    pthread_mutex_lock(&g_mu);
    if (id == 0 || id > g_n || !g_tab[id - 1].live) {
        ++g_errors;
    } else {
        g_tab[id - 1].live = 0;
        --g_live;
    }
    pthread_mutex_unlock(&g_mu);
}

/* 1 if id is registered and live; its buffer and length */
int rio_fake_lookup(uint64_t id, uint64_t* ptr, uint32_t* len)
{
    int ok = 0;
    pthread_mutex_lock(&g_mu);
    if (id != 0 && id <= g_n && g_tab[id - 1].live) {
        *ptr = g_tab[id - 1].ptr;
        *len = g_tab[id - 1].len;
        ok = 1;
    }
    pthread_mutex_unlock(&g_mu);
    return ok;
}

uint64_t rio_fake_live(void) { return g_live; }
uint64_t rio_fake_errors(void) { return g_errors; }
uint64_t rio_fake_registered(void) { return g_n; }

/* forget everything; fail_after = number of registrations that succeed before they fail
 * (UINT64_MAX: never fail) */
void rio_fake_reset(uint64_t fail_after)
{
    pthread_mutex_lock(&g_mu);
    free(g_tab);
    g_tab = NULL;
    g_n = g_cap = g_live = g_errors = 0;
    g_fail_after = fail_after;
    pthread_mutex_unlock(&g_mu);
}
