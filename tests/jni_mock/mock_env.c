/*
 * mock_env.c -- a mock JNI environment for rs_jni_core.c (TEST ONLY).
 *
 * Java arrays are heap objects (byte[], boolean[], Object[]).  The mock keeps
 * the books a real JVM would enforce with -Xcheck:jni:
 *   - local references: live count, high-water mark, the capacity the code
 *     ensured (a native frame gets 16 without EnsureLocalCapacity);
 *   - critical regions: open count, and every JNI call made while one is open
 *     (illegal) is counted as a violation;
 *   - a pending exception: class and message; JNI calls other than
 *     ExceptionCheck / DeleteLocalRef / releases with one pending are counted
 *     as violations too;
 *   - region copies in and out (bytes), to tell the pinned and staged paths apart;
 *   - with mock_moving(1), a compacting GC: every critical get of an array
 *     no region holds moves it to a fresh mapping and unmaps the old one, so
 *     an access through an address from an earlier region faults.
 * It also provides a fake coding backend (codes out[p][b] = XOR_i in[i][b] ^
 * (p + 1), checks nothing but pointers) so the CPU tests see data movement;
 * it honours a relocator (rs_set_relocator) as librsamd does, pinning the
 * arrays once around each fake call.
 */
#define _DEFAULT_SOURCE /* MAP_ANONYMOUS under -std=c11 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include "rs_jni_core.h"

enum { K_BYTES = 1, K_BOOLS = 2, K_OBJECTS = 3, K_DIRECT = 4 };

typedef struct mobj {
    int kind, len;
    uint8_t *data;        /* bytes / booleans (mapped: alloc_data) */
    struct mobj **elems;  /* objects */
    int pins;             /* open critical regions on it */
} mobj;

typedef struct {
    int live_refs, max_live_refs, capacity;
    int critical_open, max_critical_open;
    int violations;
    int exc;
    char exc_cls[128], exc_msg[512];
    long long bytes_in, bytes_out, critical_gets, commits, aborts;
    int fail_critical;     /* critical_get returns NULL when set */
    int force_copy;        /* critical_get reports isCopy (the data is still the array's) */
    int moving;            /* critical_get moves an unpinned array first */
    long long moves;
} mstate;

static mstate S;

/* ---- objects (exported to the Python test) ---- */

/* Java arrays' pages: 4 KiB (a JVM heap by default) or, with
 * mock_hugepages(1), transparent huge pages (-XX:+UseTransparentHugePages). */
static int huge_pages;
void mock_hugepages(int on) { huge_pages = on; }

static size_t map_bytes(int len) { return ((size_t)(len > 0 ? len : 1) + 4095) & ~(size_t)4095; }
static uint8_t *alloc_data(int len) {  /* zeroed */
    void *p = mmap(NULL, map_bytes(len), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return NULL;
    madvise(p, map_bytes(len), huge_pages ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
    return (uint8_t *)p;
}

mobj *mock_new_bytes(int len) {
    mobj *o = (mobj *)calloc(1, sizeof *o);
    o->kind = K_BYTES;
    o->len = len;
    o->data = alloc_data(len);
    return o;
}
mobj *mock_new_bools(int len) {
    mobj *o = mock_new_bytes(len);
    o->kind = K_BOOLS;
    return o;
}
mobj *mock_new_objects(int len) {
    mobj *o = (mobj *)calloc(1, sizeof *o);
    o->kind = K_OBJECTS;
    o->len = len;
    o->elems = (mobj **)calloc((size_t)(len > 0 ? len : 1), sizeof(mobj *));
    return o;
}
/* a direct ByteBuffer over caller memory (data not owned) */
mobj *mock_new_direct(uint8_t *p, int cap) {
    mobj *o = (mobj *)calloc(1, sizeof *o);
    o->kind = K_DIRECT;
    o->len = cap;
    o->data = p;
    return o;
}
void mock_set(mobj *outer, int i, mobj *inner) { outer->elems[i] = inner; }
uint8_t *mock_data(mobj *o) { return o->data; }
void mock_reset(void) {
    const int moving = S.moving;
    memset(&S, 0, sizeof S);
    S.capacity = 16;
    S.moving = moving;
}
void mock_fail_critical(int on) { S.fail_critical = on; }
void mock_force_copy(int on) { S.force_copy = on; }
void mock_moving(int on) { S.moving = on; }
long long mock_moves(void) { return S.moves; }
const char *mock_exc_class(void) { return S.exc ? S.exc_cls : ""; }
const char *mock_exc_message(void) { return S.exc ? S.exc_msg : ""; }
void mock_stats(long long *out) {
    out[0] = S.live_refs;
    out[1] = S.max_live_refs;
    out[2] = S.capacity;
    out[3] = S.critical_open;
    out[4] = S.max_critical_open;
    out[5] = S.violations;
    out[6] = S.bytes_in;
    out[7] = S.bytes_out;
    out[8] = S.critical_gets;
    out[9] = S.commits;
    out[10] = S.aborts;
}

/* ---- rsj_env over the mock ---- */

static void jni_call(int allowed_with_exception) {
    if (S.critical_open) S.violations++;
    if (S.exc && !allowed_with_exception) S.violations++;
}

static int m_array_length(rsj_env *e, rsj_obj a) {
    jni_call(0);
    return ((mobj *)a)->len;
}
static rsj_obj m_object_element(rsj_env *e, rsj_obj a, int i) {
    jni_call(0);
    mobj *o = (mobj *)a;
    if (i < 0 || i >= o->len) {
        S.exc = 1;
        strcpy(S.exc_cls, "java/lang/ArrayIndexOutOfBoundsException");
        strcpy(S.exc_msg, "GetObjectArrayElement");
        return NULL;
    }
    if (!o->elems[i]) return NULL;
    S.live_refs++;
    if (S.live_refs > S.max_live_refs) S.max_live_refs = S.live_refs;
    if (S.live_refs > S.capacity) S.violations++;
    return o->elems[i];
}
static void m_delete_local(rsj_env *e, rsj_obj o) {
    jni_call(1);
    S.live_refs--;
}
static int m_ensure_local_capacity(rsj_env *e, int n) {
    jni_call(0);
    if (S.live_refs + n > S.capacity) S.capacity = S.live_refs + n;
    return 0;
}
static uint8_t *m_critical_get(rsj_env *e, rsj_obj a, int *is_copy) {
    if (S.exc) S.violations++;
    *is_copy = S.force_copy;
    if (S.fail_critical) return NULL;
    mobj *o = (mobj *)a;
    if (S.moving && o->kind != K_DIRECT && o->pins == 0) {  /* the GC moved it since the last region */
        uint8_t *to = alloc_data(o->len);
        if (!to) return NULL;
        memcpy(to, o->data, (size_t)(o->len > 0 ? o->len : 0));
        munmap(o->data, map_bytes(o->len));
        o->data = to;
        S.moves++;
    }
    o->pins++;
    S.critical_open++;
    S.critical_gets++;
    if (S.critical_open > S.max_critical_open) S.max_critical_open = S.critical_open;
    return o->data;
}
static void m_critical_release(rsj_env *e, rsj_obj a, uint8_t *p, int mode) {
    mobj *o = (mobj *)a;
    if (p != o->data) S.violations++;  /* released with an address it no longer has */
    o->pins--;
    S.critical_open--;
    if (mode == RSJ_COMMIT) S.commits++;
    else S.aborts++;
}
static void bounds(mobj *o, int start, int len) {
    if (start < 0 || len < 0 || start + len > o->len) {
        S.exc = 1;
        strcpy(S.exc_cls, "java/lang/ArrayIndexOutOfBoundsException");
        strcpy(S.exc_msg, "region");
    }
}
static void m_byte_region_get(rsj_env *e, rsj_obj a, int start, int len, uint8_t *dst) {
    jni_call(0);
    mobj *o = (mobj *)a;
    bounds(o, start, len);
    if (S.exc) return;
    memcpy(dst, o->data + start, (size_t)len);
    S.bytes_in += len;
}
static void m_byte_region_set(rsj_env *e, rsj_obj a, int start, int len, const uint8_t *src) {
    jni_call(0);
    mobj *o = (mobj *)a;
    bounds(o, start, len);
    if (S.exc) return;
    memcpy(o->data + start, src, (size_t)len);
    S.bytes_out += len;
}
static void m_bool_region_get(rsj_env *e, rsj_obj a, int start, int len, uint8_t *dst) {
    m_byte_region_get(e, a, start, len, dst);
}
static int m_exception_pending(rsj_env *e) {
    if (S.critical_open) S.violations++;
    return S.exc;
}
static void m_throw_new(rsj_env *e, const char *cls, const char *msg) {
    jni_call(0);
    S.exc = 1;
    strncpy(S.exc_cls, cls, sizeof S.exc_cls - 1);
    strncpy(S.exc_msg, msg ? msg : "", sizeof S.exc_msg - 1);
}

static uint8_t *m_direct_address(rsj_env *e, rsj_obj b) {
    jni_call(0);
    return ((mobj *)b)->kind == K_DIRECT ? ((mobj *)b)->data : NULL;
}
static int64_t m_direct_capacity(rsj_env *e, rsj_obj b) {
    jni_call(0);
    return ((mobj *)b)->kind == K_DIRECT ? ((mobj *)b)->len : -1;
}
static rsj_obj m_new_direct(rsj_env *e, void *p, int64_t cap) {
    jni_call(0);
    S.live_refs++; /* the returned local reference (the Java caller takes it over) */
    if (S.live_refs > S.max_live_refs) S.max_live_refs = S.live_refs;
    return mock_new_direct((uint8_t *)p, (int)cap);
}

static rsj_env ENV = {NULL,           m_array_length,    m_object_element,   m_delete_local,
                      m_ensure_local_capacity, m_critical_get, m_critical_release, m_byte_region_get,
                      m_byte_region_set, m_bool_region_get, m_exception_pending, m_throw_new,
                      m_direct_address, m_direct_capacity, m_new_direct};

/* ---- fake backend: real argument checks from librsamd, fake coding ---- */

static int fake_data_shards(const rs_codec *c) { return rs_codec_data_shard_count(c); }

/* A relocator set on the fake backend (as librsamd keeps one per thread): the
 * fake calls pin the arrays once around their work and use the addresses the
 * acquire gave, moving every argument that lies in a key range. */
static struct {
    int on;
    rs_relocator r;
    uint8_t *base[2 * RSJ_MAX_SHARDS + 1];
    int failed;
} REL;
static int fake_set_relocator(const rs_relocator *r) {
    REL.on = r != NULL;
    if (r) REL.r = *r;
    return 0;
}
static int rel_begin(void) {
    if (!REL.on) return 0;
    if (REL.r.acquire(REL.r.user, REL.base)) return RS_E_INVALID;
    return 0;
}
static void rel_end(void) {
    if (REL.on) REL.r.release(REL.r.user, REL.base);
}
static uint8_t *rel(const uint8_t *p) {
    if (!REL.on || !p) return (uint8_t *)p;
    for (int i = 0; i < REL.r.n; i++) {
        const uintptr_t k = (uintptr_t)REL.r.keys[i], a = (uintptr_t)p;
        if (a >= k && a - k <= (uintptr_t)REL.r.lens[i]) return REL.base[i] + (a - k);
    }
    return (uint8_t *)p;
}
/* sh[0..n) moved into out[] */
static uint8_t **rel_all(const uint8_t *const *sh, int n, uint8_t **out) {
    for (int i = 0; i < n; i++) out[i] = rel(sh[i]);
    return out;
}

static void enc_raw(int k, uint8_t *const *sh, int n, int32_t off, int32_t cnt) {
    for (int p = k; p < n; p++)
        for (int32_t b = off; b < off + cnt; b++) {
            uint8_t x = (uint8_t)(p - k + 1);
            for (int i = 0; i < k; i++) x ^= sh[i][b];
            sh[p][b] = x;
        }
}
/* missing shard j := XOR of the present shards ^ 0x80 ^ j (data movement only) */
static void dec_raw(uint8_t *const *sh, int n, const uint8_t *pres, int32_t off, int32_t cnt) {
    for (int j = 0; j < n; j++) {
        if (pres[j]) continue;
        for (int32_t b = off; b < off + cnt; b++) {
            uint8_t x = (uint8_t)(0x80 ^ j);
            for (int i = 0; i < n; i++)
                if (pres[i]) x ^= sh[i][b];
            sh[j][b] = x;
        }
    }
}

static int fake_encode(const rs_codec *c, uint8_t *const *sh, int n, const int64_t *lens, int32_t off, int32_t cnt) {
    int rc = rs_check_buffers_and_sizes(c, n, lens, off, cnt);
    if (rc || cnt <= 0) return rc;
    if ((rc = rel_begin())) return rc;
    uint8_t *p[RSJ_MAX_SHARDS];
    enc_raw(rs_codec_data_shard_count(c), rel_all((const uint8_t *const *)sh, n, p), n, off, cnt);
    rel_end();
    return 0;
}
static int fake_decode(const rs_codec *c, uint8_t *const *sh, int n, const int64_t *lens, const uint8_t *pres,
                       int32_t off, int32_t cnt) {
    int rc = rs_check_buffers_and_sizes(c, n, lens, off, cnt);
    if (rc || cnt <= 0) return rc;
    if ((rc = rel_begin())) return rc;
    uint8_t *p[RSJ_MAX_SHARDS];
    dec_raw(rel_all((const uint8_t *const *)sh, n, p), n, pres, off, cnt);
    rel_end();
    return 0;
}
static int fake_verify(const rs_codec *c, uint8_t *const *sh, int n, const int64_t *lens, int32_t off, int32_t cnt,
                       const uint8_t *temp, int64_t temp_len, int *result) {
    int rc = rs_check_buffers_and_sizes(c, n, lens, off, cnt);
    if (rc) return rc;
    if (temp && temp_len < (int64_t)off + cnt) return RS_E_TEMP_TOO_SMALL;
    *result = 1;
    if (cnt <= 0) return 0;
    if ((rc = rel_begin())) return rc;
    uint8_t *q[RSJ_MAX_SHARDS];
    uint8_t *const *v = rel_all((const uint8_t *const *)sh, n, q);
    const int k = rs_codec_data_shard_count(c);
    for (int p = k; p < n && *result; p++)
        for (int32_t b = off; b < off + cnt; b++) {
            uint8_t x = (uint8_t)(p - k + 1);
            for (int i = 0; i < k; i++) x ^= v[i][b];
            if (v[p][b] != x) {
                *result = 0;
                break;
            }
        }
    rel_end();
    return 0;
}
static int fake_code(const uint8_t *const *rows, const uint8_t *const *in, int nin, uint8_t *const *out, int nout,
                     int32_t off, int32_t cnt) {
    int rc = rel_begin();
    if (rc) return rc;
    uint8_t *ip[RSJ_MAX_SHARDS], *op[RSJ_MAX_SHARDS];
    rel_all(in, nin, ip);
    rel_all((const uint8_t *const *)out, nout, op);
    for (int p = 0; p < nout; p++)
        for (int32_t b = off; b < off + cnt; b++) {
            uint8_t x = 0;
            for (int i = 0; i < nin; i++) x ^= (uint8_t)(ip[i][b] + rows[p][i]);
            op[p][b] = x;
        }
    rel_end();
    return 0;
}
static int fake_check(const uint8_t *const *rows, const uint8_t *const *in, int nin, const uint8_t *const *chk,
                      int nchk, int32_t off, int32_t cnt, int *result) {
    int rc = rel_begin();
    if (rc) return rc;
    uint8_t *ip[RSJ_MAX_SHARDS], *cp[RSJ_MAX_SHARDS];
    rel_all(in, nin, ip);
    rel_all(chk, nchk, cp);
    *result = 1;
    for (int p = 0; p < nchk; p++)
        for (int32_t b = off; b < off + cnt; b++) {
            uint8_t x = 0;
            for (int i = 0; i < nin; i++) x ^= (uint8_t)(ip[i][b] + rows[p][i]);
            if (cp[p][b] != x) *result = 0;
        }
    rel_end();
    return 0;
}

/* shard-major recovery: records its arguments and the flags it was handed */
static struct {
    const rs_codec *c;
    uint64_t base, stride, chunk, n;
    void *stream;
    uint8_t flags[4096];
    int rc;
} SM;
static int fake_shard_major(const rs_codec *c, uint8_t *base, size_t stride, size_t chunk, size_t n,
                            const uint8_t *present, void *stream) {
    SM.c = c;
    SM.base = (uint64_t)(uintptr_t)base;
    SM.stride = stride;
    SM.chunk = chunk;
    SM.n = n;
    SM.stream = stream;
    const size_t nf = n * (size_t)rs_codec_total_shard_count(c);
    memcpy(SM.flags, present, nf < sizeof SM.flags ? nf : sizeof SM.flags);
    return SM.rc;
}

/* file layout: the real split / merge (ReedSolomonEncoder.java:62-74,
 * ReedSolomonDecoder.java:92-103) around the fake parity and decode above;
 * every call's file length and first shard length are recorded */
static struct {
    int calls;
    int64_t file_len[64], shard_len[64];
} FC;
static void file_record(int64_t flen, int64_t slen) {
    if (FC.calls < 64) {
        FC.file_len[FC.calls] = flen;
        FC.shard_len[FC.calls] = slen;
    }
    FC.calls++;
}
static int fake_file_encode(const rs_codec *c, const uint8_t *file, int64_t flen, int32_t block, uint8_t *const *sh,
                            int n, const int64_t *lens) {
    int64_t padded = 0, S = 0;
    int rc = rs_file_layout(c, flen, block, &padded, &S);
    if (rc) return rc;
    file_record(flen, n ? lens[0] : -1);
    rc = rs_check_buffers_and_sizes(c, n, lens, 0, S);
    if (rc) return rc;
    if ((rc = rel_begin())) return rc;
    uint8_t *p[RSJ_MAX_SHARDS];
    uint8_t *const *v = rel_all((const uint8_t *const *)sh, n, p);
    const uint8_t *f = rel(file);
    const int k = rs_codec_data_shard_count(c);
    for (int64_t blk = 0; blk < padded / block; blk++)
        for (int32_t i = 0; i < block; i++) {
            const int64_t at = blk * block + i;
            v[blk % k][(blk / k) * block + i] = at < flen ? f[at] : 0;
        }
    enc_raw(k, v, n, 0, (int32_t)S);
    rel_end();
    return 0;
}
static int fake_file_decode(const rs_codec *c, uint8_t *const *sh, int n, const int64_t *lens, const uint8_t *pres,
                            int32_t cnt, int32_t block, uint8_t *out, int64_t fsize) {
    int rc = rs_check_buffers_and_sizes(c, n, lens, 0, cnt);
    if (rc) return rc;
    const int k = rs_codec_data_shard_count(c);
    int np = 0;
    for (int i = 0; i < n; i++) np += pres[i] ? 1 : 0;
    if (np < k) return RS_E_NOT_ENOUGH;
    if (block < 1 || lens[0] % block || fsize < 0 || fsize > k * lens[0]) return RS_E_INVALID;
    file_record(fsize, lens[0]);
    if ((rc = rel_begin())) return rc;
    uint8_t *p[RSJ_MAX_SHARDS];
    uint8_t *const *v = rel_all((const uint8_t *const *)sh, n, p);
    uint8_t *o = rel(out);
    if (np < n && cnt > 0) dec_raw(v, n, pres, 0, cnt);
    for (int64_t at = 0; at < fsize; at++) {
        const int64_t blk = at / block;
        o[at] = v[blk % k][(blk / k) * block + at % block];
    }
    rel_end();
    return 0;
}
/* the master's host arrays: every absent chunk of group g := the fake decode
 * of that group's chunks (checks as librsamd: count, lengths, >= k present) */
static int fake_shard_major_host(const rs_codec *c, uint8_t *const *sv, int n, const int64_t *lens, size_t chunk,
                                 size_t groups, const uint8_t *pres) {
    const int T = rs_codec_total_shard_count(c), k = rs_codec_data_shard_count(c);
    if (n != T) return RS_E_WRONG_NSHARDS;
    for (int s = 0; s < n; s++)
        if (lens[s] < (int64_t)(chunk * groups)) return RS_E_INVALID;
    for (size_t g = 0; g < groups; g++) {
        int np = 0;
        for (int s = 0; s < n; s++) np += pres[g * n + s] ? 1 : 0;
        if (np < k) return RS_E_NOT_ENOUGH;
    }
    int rc = rel_begin();
    if (rc) return rc;
    uint8_t *p[RSJ_MAX_SHARDS];
    uint8_t *const *v = rel_all((const uint8_t *const *)sv, n, p);
    for (size_t g = 0; g < groups; g++) {
        uint8_t *at[RSJ_MAX_SHARDS];
        for (int s = 0; s < n; s++) at[s] = v[s] + g * chunk;
        dec_raw(at, n, pres + g * n, 0, (int32_t)chunk);
    }
    rel_end();
    return 0;
}
/* pinned host memory: plain malloc, counted */
static int host_live;
static int fake_host_alloc(void **out, size_t n) {
    *out = malloc(n ? n : 1);
    if (!*out) return RS_E_HIP;
    host_live++;
    return 0;
}
static int fake_host_free(void *p) {
    free(p);
    host_live--;
    return 0;
}
int mock_host_live(void) { return host_live; }
void mock_file_record(int64_t *out, int max) {
    out[0] = FC.calls;
    for (int i = 0; i < FC.calls && i < 64 && 2 * i + 2 < max; i++) {
        out[1 + 2 * i] = FC.file_len[i];
        out[2 + 2 * i] = FC.shard_len[i];
    }
    FC.calls = 0;
}

static const rsj_backend FAKE = {fake_encode,       fake_decode,         fake_verify,
                                 fake_code,         fake_check,          rs_check_buffers_and_sizes,
                                 rs_codec_total_shard_count, fake_data_shards, rs_last_error_message,
                                 fake_shard_major,  rs_file_layout,      fake_file_encode,
                                 fake_file_decode,  fake_host_alloc,     fake_host_free,
                                 fake_shard_major_host, fake_set_relocator};

static const rsj_backend *backend(int real) { return real ? rsj_librsamd_backend() : &FAKE; }

/* ---- entry points for the Python test (backend: 0 fake, 1 librsamd) ---- */

void mock_encode_parity(int real, const rs_codec *c, mobj *shards, int32_t off, int32_t cnt) {
    rsj_encode_parity(&ENV, backend(real), c, shards, off, cnt);
}
void mock_decode_missing(int real, const rs_codec *c, mobj *shards, mobj *present, int32_t off, int32_t cnt) {
    rsj_decode_missing(&ENV, backend(real), c, shards, present, off, cnt);
}
int mock_is_parity_correct(int real, const rs_codec *c, mobj *shards, int32_t first, int32_t cnt, mobj *temp) {
    return rsj_is_parity_correct(&ENV, backend(real), c, shards, first, cnt, temp);
}
void mock_code_some_shards(int real, mobj *rows, mobj *in, int32_t nin, mobj *out, int32_t nout, int32_t off,
                           int32_t cnt) {
    rsj_code_some_shards(&ENV, backend(real), rows, in, nin, out, nout, off, cnt);
}
int mock_check_some_shards(int real, mobj *rows, mobj *in, int32_t nin, mobj *chk, int32_t nchk, int32_t off,
                           int32_t cnt) {
    return rsj_check_some_shards(&ENV, backend(real), rows, in, nin, chk, nchk, off, cnt);
}
void mock_recover_groups_shard_major(int real, const rs_codec *c, int64_t base, int64_t stride, int32_t chunk,
                                     int64_t n, mobj *present, int64_t stream) {
    rsj_recover_groups_shard_major(&ENV, backend(real), c, base, stride, chunk, n, present, stream);
}
/* the fake's record: out[0..4] = base, stride, chunk, n, stream; flags copied to `flags` */
void mock_shard_major_record(uint64_t *out, uint8_t *flags, int nflags) {
    out[0] = SM.base;
    out[1] = SM.stride;
    out[2] = SM.chunk;
    out[3] = SM.n;
    out[4] = (uint64_t)(uintptr_t)SM.stream;
    memcpy(flags, SM.flags, nflags < (int)sizeof SM.flags ? (size_t)nflags : sizeof SM.flags);
}
void mock_shard_major_rc(int rc) { SM.rc = rc; }
void mock_file_encode(int real, const rs_codec *c, mobj *file, int32_t block, mobj *shards) {
    rsj_file_encode(&ENV, backend(real), c, file, block, shards);
}
void mock_file_decode(int real, const rs_codec *c, mobj *shards, mobj *present, int32_t cnt, int32_t block, mobj *out,
                      int32_t fsize) {
    rsj_file_decode(&ENV, backend(real), c, shards, present, cnt, block, out, fsize);
}
mobj *mock_alloc_pinned(int real, int32_t cap) { return (mobj *)rsj_alloc_pinned(&ENV, backend(real), cap); }
void mock_free_pinned(int real, mobj *buf) { rsj_free_pinned(&ENV, backend(real), buf); }
/* the Java caller dropping its local reference to a buffer from new_direct */
void mock_drop_local(void) { S.live_refs--; }
void mock_encode_parity_direct(int real, const rs_codec *c, mobj *shards, int32_t off, int32_t cnt) {
    rsj_encode_parity_direct(&ENV, backend(real), c, shards, off, cnt);
}
void mock_decode_missing_direct(int real, const rs_codec *c, mobj *shards, mobj *present, int32_t off, int32_t cnt) {
    rsj_decode_missing_direct(&ENV, backend(real), c, shards, present, off, cnt);
}
void mock_file_encode_direct(int real, const rs_codec *c, mobj *file, int32_t flen, int32_t block, mobj *shards) {
    rsj_file_encode_direct(&ENV, backend(real), c, file, flen, block, shards);
}
void mock_file_decode_direct(int real, const rs_codec *c, mobj *shards, mobj *present, int32_t cnt, int32_t block,
                             mobj *out, int32_t fsize) {
    rsj_file_decode_direct(&ENV, backend(real), c, shards, present, cnt, block, out, fsize);
}
void mock_recover_groups_shard_major_host(int real, const rs_codec *c, mobj *servers, int32_t chunk, int32_t n,
                                          mobj *present) {
    rsj_recover_groups_shard_major_host(&ENV, backend(real), c, servers, chunk, n, present);
}
void mock_recover_groups_shard_major_direct(int real, const rs_codec *c, mobj *servers, int32_t chunk, int32_t n,
                                            mobj *present) {
    rsj_recover_groups_shard_major_direct(&ENV, backend(real), c, servers, chunk, n, present);
}

/* ---- timing loops for bench.py's host legs (a C caller: no Python per call) ----
 * Median microseconds per call over `reps` calls after 20 warm-up calls.
 * kind: 0 encodeParity, 1 decodeMissing.  mock_time_jni goes through the JNI
 * core (rsj_* over this mock JNIEnv, the real backend), mock_time_capi calls
 * the C-ABI directly. */
#include <time.h>

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp_double(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

static double median_of(double *t, int n) {
    qsort(t, (size_t)n, sizeof *t, cmp_double);
    return t[n / 2];
}

double mock_time_jni(int kind, const rs_codec *c, mobj *shards, mobj *present, int32_t cnt, int reps) {
    double *t = (double *)malloc(sizeof(double) * (size_t)(reps > 0 ? reps : 1));
    for (int i = -20; i < reps; i++) {
        const double t0 = now_us();
        if (kind == 0)
            rsj_encode_parity(&ENV, rsj_librsamd_backend(), c, shards, 0, cnt);
        else
            rsj_decode_missing(&ENV, rsj_librsamd_backend(), c, shards, present, 0, cnt);
        if (S.exc) {
            free(t);
            return -1.0;
        }
        if (i >= 0) t[i] = now_us() - t0;
    }
    const double m = median_of(t, reps);
    free(t);
    return m;
}

double mock_time_capi(int kind, const rs_codec *c, uint8_t *const *sh, int n, const int64_t *lens,
                      const uint8_t *present, int32_t cnt, int reps) {
    double *t = (double *)malloc(sizeof(double) * (size_t)(reps > 0 ? reps : 1));
    for (int i = -20; i < reps; i++) {
        const double t0 = now_us();
        const int rc = kind == 0 ? rs_encode_parity(c, sh, n, lens, 0, cnt)
                                 : rs_decode_missing(c, sh, n, lens, present, 0, cnt);
        if (rc) {
            free(t);
            return -1.0;
        }
        if (i >= 0) t[i] = now_us() - t0;
    }
    const double m = median_of(t, reps);
    free(t);
    return m;
}

/* The client's file calls on a small file: kind 0 rs_file_encode (file ->
 * shards), 1 rs_file_decode (shards with `present` -> out, byteCntInShard =
 * the shard length). */
double mock_time_capi_file(int kind, const rs_codec *c, const uint8_t *file, int64_t flen, int32_t block,
                           uint8_t *const *sh, int n, const int64_t *lens, const uint8_t *present, uint8_t *out,
                           int reps) {
    double *t = (double *)malloc(sizeof(double) * (size_t)(reps > 0 ? reps : 1));
    for (int i = -20; i < reps; i++) {
        const double t0 = now_us();
        const int rc = kind == 0 ? rs_file_encode(c, file, flen, block, sh, n, lens)
                                 : rs_file_decode(c, sh, n, lens, present, (int32_t)lens[0], block, out, flen);
        if (rc) {
            free(t);
            return -1.0;
        }
        if (i >= 0) t[i] = now_us() - t0;
    }
    const double m = median_of(t, reps);
    free(t);
    return m;
}
