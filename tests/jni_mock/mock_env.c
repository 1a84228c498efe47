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
 *   - region copies in and out (bytes), to tell the pinned and staged paths apart.
 * It also provides a fake coding backend (codes out[p][b] = XOR_i in[i][b] ^
 * (p + 1), checks nothing but pointers) so the CPU tests see data movement.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rs_jni_core.h"

enum { K_BYTES = 1, K_BOOLS = 2, K_OBJECTS = 3, K_DIRECT = 4 };

typedef struct mobj {
    int kind, len;
    uint8_t *data;        /* bytes / booleans */
    struct mobj **elems;  /* objects */
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
} mstate;

static mstate S;

/* ---- objects (exported to the Python test) ---- */

mobj *mock_new_bytes(int len) {
    mobj *o = (mobj *)calloc(1, sizeof *o);
    o->kind = K_BYTES;
    o->len = len;
    o->data = (uint8_t *)calloc((size_t)(len > 0 ? len : 1), 1);
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
void mock_reset(void) { memset(&S, 0, sizeof S); S.capacity = 16; }
void mock_fail_critical(int on) { S.fail_critical = on; }
void mock_force_copy(int on) { S.force_copy = on; }
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
    S.critical_open++;
    S.critical_gets++;
    if (S.critical_open > S.max_critical_open) S.max_critical_open = S.critical_open;
    return ((mobj *)a)->data;
}
static void m_critical_release(rsj_env *e, rsj_obj a, uint8_t *p, int mode) {
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

static int fake_encode(const rs_codec *c, uint8_t *const *sh, int n, const int64_t *lens, int32_t off, int32_t cnt) {
    int rc = rs_check_buffers_and_sizes(c, n, lens, off, cnt);
    if (rc) return rc;
    const int k = rs_codec_data_shard_count(c);
    for (int p = k; p < n; p++)
        for (int32_t b = off; b < off + cnt; b++) {
            uint8_t x = (uint8_t)(p - k + 1);
            for (int i = 0; i < k; i++) x ^= sh[i][b];
            sh[p][b] = x;
        }
    return 0;
}
static int fake_decode(const rs_codec *c, uint8_t *const *sh, int n, const int64_t *lens, const uint8_t *pres,
                       int32_t off, int32_t cnt) {
    int rc = rs_check_buffers_and_sizes(c, n, lens, off, cnt);
    if (rc) return rc;
    /* missing shard j := XOR of the present shards ^ 0x80 ^ j (data movement only) */
    for (int j = 0; j < n; j++) {
        if (pres[j]) continue;
        for (int32_t b = off; b < off + cnt; b++) {
            uint8_t x = (uint8_t)(0x80 ^ j);
            for (int i = 0; i < n; i++)
                if (pres[i]) x ^= sh[i][b];
            sh[j][b] = x;
        }
    }
    return 0;
}
static int fake_verify(const rs_codec *c, uint8_t *const *sh, int n, const int64_t *lens, int32_t off, int32_t cnt,
                       const uint8_t *temp, int64_t temp_len, int *result) {
    int rc = rs_check_buffers_and_sizes(c, n, lens, off, cnt);
    if (rc) return rc;
    const int k = rs_codec_data_shard_count(c);
    *result = 1;
    for (int p = k; p < n && *result; p++)
        for (int32_t b = off; b < off + cnt; b++) {
            uint8_t x = (uint8_t)(p - k + 1);
            for (int i = 0; i < k; i++) x ^= sh[i][b];
            if (sh[p][b] != x) {
                *result = 0;
                break;
            }
        }
    return 0;
}
static int fake_code(const uint8_t *const *rows, const uint8_t *const *in, int nin, uint8_t *const *out, int nout,
                     int32_t off, int32_t cnt) {
    for (int p = 0; p < nout; p++)
        for (int32_t b = off; b < off + cnt; b++) {
            uint8_t x = 0;
            for (int i = 0; i < nin; i++) x ^= (uint8_t)(in[i][b] + rows[p][i]);
            out[p][b] = x;
        }
    return 0;
}
static int fake_check(const uint8_t *const *rows, const uint8_t *const *in, int nin, const uint8_t *const *chk,
                      int nchk, int32_t off, int32_t cnt, int *result) {
    *result = 1;
    for (int p = 0; p < nchk; p++)
        for (int32_t b = off; b < off + cnt; b++) {
            uint8_t x = 0;
            for (int i = 0; i < nin; i++) x ^= (uint8_t)(in[i][b] + rows[p][i]);
            if (chk[p][b] != x) *result = 0;
        }
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
    const int k = rs_codec_data_shard_count(c);
    for (int64_t blk = 0; blk < padded / block; blk++)
        for (int32_t i = 0; i < block; i++) {
            const int64_t at = blk * block + i;
            sh[blk % k][(blk / k) * block + i] = at < flen ? file[at] : 0;
        }
    return fake_encode(c, sh, n, lens, 0, (int32_t)S);
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
    if (np < n) fake_decode(c, sh, n, lens, pres, 0, cnt);
    for (int64_t at = 0; at < fsize; at++) {
        const int64_t blk = at / block;
        out[at] = sh[blk % k][(blk / k) * block + at % block];
    }
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
                                 fake_file_decode,  fake_host_alloc,     fake_host_free};

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
