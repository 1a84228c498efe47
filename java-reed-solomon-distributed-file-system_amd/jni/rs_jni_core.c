/*
 * rs_jni_core.c -- see rs_jni_core.h.
 *
 * How a call reaches the GPU: ONE library call per Java call, with the Java
 * arrays movable (rs_set_relocator, include/rs_amd.h).  The library touches
 * caller memory only in copy batches (a chunk's inputs into its pinned slots,
 * outputs back, a file's rows split or merged), and brackets each batch with
 * this shim's acquire -- every array pinned with GetPrimitiveArrayCritical,
 * its current address handed over -- and release (outputs with mode 0, inputs
 * with JNI_ABORT).  So no critical region lasts longer than one batch's host
 * copies (about a millisecond; the GPU codes between batches with every array
 * released, and the GC may move them then), the library's pipeline runs the
 * whole range without a restart, and the shim itself copies no byte.  The
 * call's array arguments are stand-in keys (non-canonical addresses the
 * library never dereferences).
 *
 * If the JVM answers a critical get with a COPY (isCopy, seen by one probing
 * pin before the call), pinning per batch would copy whole arrays each time:
 * the call then copies slices of RSJ_SLICE_BYTES through C buffers with
 * Get/SetByteArrayRegion instead, validated up front (same checks and order
 * as the reference) so a later slice never fails after an earlier one was
 * written.  No JNI call is made while a critical region is open.  Element
 * references of the byte[][] arrays are local references: capacity is ensured
 * up front and each one is deleted before returning.
 */
#include "rs_jni_core.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NPE "java/lang/NullPointerException"
#define IAE "java/lang/IllegalArgumentException"
#define ISE "java/lang/IllegalStateException"
#define AIOOBE "java/lang/ArrayIndexOutOfBoundsException"

const rsj_backend *rsj_librsamd_backend(void) {
    static const rsj_backend b = {rs_encode_parity,           rs_decode_missing,         rs_is_parity_correct,
                                  rs_code_some_shards,        rs_check_some_shards,      rs_check_buffers_and_sizes,
                                  rs_codec_total_shard_count, rs_codec_data_shard_count, rs_last_error_message,
                                  rs_decode_groups_shard_major_dev, rs_file_layout,          rs_file_encode,
                                  rs_file_decode,             rs_host_alloc,             rs_host_free,
                                  rs_decode_groups_shard_major, rs_set_relocator};
    return &b;
}

static void throw_rc(rsj_env *e, const rsj_backend *b, int rc) {
    e->throw_new(e, (rc == RS_E_HIP || rc == RS_E_NO_DEVICE) ? ISE : IAE, b->last_error());
}

/* Java's message for a[index] past the end: "Index 5 out of bounds for length 5". */
static void throw_index(rsj_env *e, int64_t index, int64_t length) {
    char msg[96];
    snprintf(msg, sizeof msg, "Index %lld out of bounds for length %lld", (long long)index, (long long)length);
    e->throw_new(e, AIOOBE, msg);
}

/* ---- byte[][] views ---- */

typedef struct {
    int n;
    rsj_obj arr[RSJ_MAX_SHARDS];
    int64_t len[RSJ_MAX_SHARDS];
} arrays;

static void drop_refs(rsj_env *e, arrays *a) {
    for (int i = 0; i < a->n; i++)
        if (a->arr[i]) e->delete_local(e, a->arr[i]);
    a->n = 0;
}

/* Takes the first n elements of a byte[][] as local references with their
 * lengths.  A null element throws NullPointerException (where Java would
 * dereference it).  Returns 0, or -1 with an exception pending. */
static int take(rsj_env *e, rsj_obj outer, int n, arrays *a) {
    a->n = 0;
    if (n > RSJ_MAX_SHARDS) n = RSJ_MAX_SHARDS;
    if (n > 0 && e->ensure_local_capacity(e, n + 4) < 0) return -1;
    for (int i = 0; i < n; i++) {
        rsj_obj x = e->object_element(e, outer, i);
        if (e->exception_pending(e)) {
            drop_refs(e, a);
            return -1;
        }
        a->arr[i] = x;
        a->n = i + 1;
        if (!x) {
            drop_refs(e, a);
            e->throw_new(e, NPE, "byte[] element is null");
            return -1;
        }
        a->len[i] = e->array_length(e, x);
    }
    return 0;
}

/* Slice buffers for the copying path: one RSJ_SLICE_BYTES buffer per array. */
static uint8_t *slice_buffers(int n, uint8_t **ptrs) {
    uint8_t *mem = (uint8_t *)malloc((size_t)(n > 0 ? n : 1) * RSJ_SLICE_BYTES);
    for (int i = 0; mem && i < n; i++) ptrs[i] = mem + (size_t)i * RSJ_SLICE_BYTES;
    return mem;
}

/* ---- movable arrays (rs_set_relocator) ---- */

/* Stand-in address of array i: non-canonical on x86-64 and aarch64, so never
 * real memory; a Java array holds < 2^31 bytes < 2^36. */
#define RSJ_KEY(i) ((uint8_t *)(uintptr_t)(0x4000000000000000ull + ((uint64_t)(i) << 36)))
#define RSJ_MAX_ARRAYS (2 * RSJ_MAX_SHARDS + 1)

typedef struct {
    rsj_env *e;
    int n;
    rsj_obj arr[RSJ_MAX_ARRAYS];
    int64_t len[RSJ_MAX_ARRAYS];
    int mode[RSJ_MAX_ARRAYS];  /* release mode after a batch: RSJ_COMMIT for written arrays */
    const uint8_t *key[RSJ_MAX_ARRAYS];
    int acquire_failed;
} movable;

static void mv_init(movable *mv, rsj_env *e) {
    mv->e = e;
    mv->n = 0;
    mv->acquire_failed = 0;
}

static void mv_add(movable *mv, rsj_obj arr, int64_t len, int mode) {
    mv->arr[mv->n] = arr;
    mv->len[mv->n] = len;
    mv->mode[mv->n] = mode;
    mv->key[mv->n] = RSJ_KEY(mv->n);
    mv->n++;
}

/* Pins every array into base[] (is_copy: whether any came back as a copy).
 * On a failed get the ones pinned are released and -1 returned. */
static int mv_pin(movable *mv, uint8_t **base, int *is_copy) {
    *is_copy = 0;
    for (int i = 0; i < mv->n; i++) {
        int c = 0;
        base[i] = mv->e->critical_get(mv->e, mv->arr[i], &c);
        *is_copy |= c;
        if (!base[i] && mv->len[i] > 0) {
            for (int j = i - 1; j >= 0; j--)
                if (base[j]) mv->e->critical_release(mv->e, mv->arr[j], base[j], RSJ_ABORT);
            return -1;
        }
    }
    return 0;
}

static void mv_unpin(movable *mv, uint8_t **base, const int *mode) {
    for (int i = mv->n - 1; i >= 0; i--)
        if (base[i]) mv->e->critical_release(mv->e, mv->arr[i], base[i], mode ? mode[i] : RSJ_ABORT);
}

static int mv_acquire(void *user, uint8_t **base) {
    movable *mv = (movable *)user;
    int c;
    if (mv_pin(mv, base, &c)) {
        mv->acquire_failed = 1;
        return -1;
    }
    return 0;
}

static void mv_release(void *user, uint8_t **base) {
    movable *mv = (movable *)user;
    mv_unpin(mv, base, mv->mode);
}

/* The probe before a call: 0 with *copies set, or -1 with OutOfMemoryError
 * pending (a critical get failed). */
static int mv_probe(movable *mv, int *copies) {
    uint8_t *base[RSJ_MAX_ARRAYS];
    if (mv_pin(mv, base, copies)) {
        mv->e->throw_new(mv->e, "java/lang/OutOfMemoryError", "GetPrimitiveArrayCritical failed");
        return -1;
    }
    mv_unpin(mv, base, NULL);
    return 0;
}

static rs_relocator mv_relocator(movable *mv) {
    rs_relocator r = {mv, mv->n, mv->key, mv->len, mv_acquire, mv_release};
    return r;
}

/* After a relocated backend call: 0, or -1 with the exception pending. */
static int mv_result(rsj_env *e, const rsj_backend *b, movable *mv, int rc) {
    if (!rc) return 0;
    if (mv->acquire_failed)
        e->throw_new(e, "java/lang/OutOfMemoryError", "GetPrimitiveArrayCritical failed");
    else
        e->throw_new(e, (rc == RS_E_HIP || rc == RS_E_NO_DEVICE) ? ISE : IAE, b->last_error());
    return -1;
}

/* ---- ReedSolomon (codec-level) natives ---- */

enum { ROLE_NONE = 0, ROLE_IN = 1, ROLE_OUT = 2 };
enum { OP_ENCODE, OP_DECODE, OP_VERIFY };

/* One slice through the backend: arrays at `ptr` with lengths `len`, bytes
 * [off, off + n) (shard-level calls; the backend re-checks the sizes). */
static int shard_slice(const rsj_backend *b, const rs_codec *c, int op, uint8_t *const *ptr, int n_arr,
                       const int64_t *len, const uint8_t *present, int32_t off, int32_t n, const uint8_t *temp,
                       int64_t temp_len, int *part) {
    *part = 1;
    if (op == OP_ENCODE) return b->encode_parity(c, ptr, n_arr, len, off, n);
    if (op == OP_DECODE) return b->decode_missing(c, ptr, n_arr, len, present, off, n);
    return b->is_parity_correct(c, ptr, n_arr, len, off, n, temp, temp_len, part);
}

/* The copying fallback (a JVM whose critical gets return copies): validated
 * up front, then slice by slice through C buffers with Get/SetByteArrayRegion
 * (only the arrays role[] says are read are copied in, only those written
 * copied out).  Returns 0 (result in *result) or -1 with an exception pending. */
static int shard_call_copying(rsj_env *e, const rsj_backend *b, const rs_codec *c, arrays *s, const int *role, int op,
                              const uint8_t *present, int32_t offset, int32_t count, const uint8_t *temp,
                              int64_t temp_len, int *result) {
    int rc = b->check_buffers_and_sizes(c, s->n, s->len, offset, count);
    if (rc) {
        throw_rc(e, b, rc);
        return -1;
    }
    if (op == OP_VERIFY && temp && temp_len < (int64_t)offset + count) {  /* ReedSolomon.java:147-151 */
        e->throw_new(e, IAE, "tempBuffer is not big enough");
        return -1;
    }
    uint8_t *buf[RSJ_MAX_SHARDS];
    uint8_t *mem = slice_buffers(s->n, buf);
    if (!mem) {
        e->throw_new(e, "java/lang/OutOfMemoryError", "slice buffers");
        return -1;
    }
    int64_t lens[RSJ_MAX_SHARDS];
    int32_t done = 0;
    do {  /* at least once: a zero-byte call still gets the backend's checks */
        const int32_t left = count - done;
        const int32_t n = left < (int32_t)RSJ_SLICE_BYTES ? left : (int32_t)RSJ_SLICE_BYTES;
        int part = 1;
        for (int i = 0; i < s->n; i++) {
            lens[i] = n;
            if (role[i] & ROLE_IN) e->byte_region_get(e, s->arr[i], offset + done, n, buf[i]);
        }
        if (e->exception_pending(e)) break;
        rc = shard_slice(b, c, op, buf, s->n, lens, present, 0, n, temp ? buf[0] : NULL, temp ? n : 0, &part);
        if (rc) {
            throw_rc(e, b, rc);
            break;
        }
        for (int i = 0; i < s->n; i++)
            if (role[i] & ROLE_OUT) e->byte_region_set(e, s->arr[i], offset + done, n, buf[i]);
        if (e->exception_pending(e)) break;
        if (!part) *result = 0; /* isParityCorrect: false at the first mismatch */
        done += n;
    } while (done < count && *result);
    free(mem);
    return e->exception_pending(e) ? -1 : 0;
}

/* The shard-array call: role[i] says whether shard i is read and/or written.
 * One backend call over the whole range with the arrays movable (the file
 * header); the copying fallback when the JVM copies.  Returns 0 (result in
 * *result) or -1 with an exception pending. */
static int shard_call(rsj_env *e, const rsj_backend *b, const rs_codec *c, arrays *s, const int *role, int op,
                      const uint8_t *present, int32_t offset, int32_t count, const uint8_t *temp, int64_t temp_len,
                      int *result) {
    *result = 1;
    if (op == OP_VERIFY && temp) {  /* checkBuffersAndSizes, then the tempBuffer (ReedSolomon.java:147-151) */
        const int rc = b->check_buffers_and_sizes(c, s->n, s->len, offset, count);
        if (rc) {
            throw_rc(e, b, rc);
            return -1;
        }
        if (temp_len < (int64_t)offset + count) {
            e->throw_new(e, IAE, "tempBuffer is not big enough");
            return -1;
        }
    }
    movable mv;
    mv_init(&mv, e);
    for (int i = 0; i < s->n; i++) mv_add(&mv, s->arr[i], s->len[i], (role[i] & ROLE_OUT) ? RSJ_COMMIT : RSJ_ABORT);
    int copies = 0;
    if (mv_probe(&mv, &copies)) return -1;
    if (copies && count > 0)
        return shard_call_copying(e, b, c, s, role, op, present, offset, count, temp, temp_len, result);
    const rs_relocator r = mv_relocator(&mv);
    b->set_relocator(&r);
    int part = 1;
    const int rc = shard_slice(b, c, op, (uint8_t *const *)mv.key, s->n, s->len, present, offset, count, temp,
                               temp_len, &part);
    b->set_relocator(NULL);
    if (mv_result(e, b, &mv, rc)) return -1;
    *result = part;
    return 0;
}

/* shards.length != totalShardCount is reported before any element is touched
 * (ReedSolomon.java:280-282); then the elements are taken. */
static int take_shards(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, arrays *s) {
    if (!shards) {
        e->throw_new(e, NPE, "shards is null");
        return -1;
    }
    const int n = e->array_length(e, shards);
    if (n != b->total_shards(c)) {
        int64_t none = 0;
        throw_rc(e, b, b->check_buffers_and_sizes(c, n, &none, 0, 0));
        return -1;
    }
    return take(e, shards, n, s);
}

void rsj_encode_parity(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, int32_t offset,
                       int32_t count) {
    arrays s;
    if (take_shards(e, b, c, shards, &s)) return;
    /* data shards are read, parity shards written (ReedSolomon.java:90-104) */
    const int k = b->data_shards(c);
    int role[RSJ_MAX_SHARDS];
    for (int i = 0; i < s.n; i++) role[i] = i < k ? ROLE_IN : ROLE_OUT;
    int result;
    shard_call(e, b, c, &s, role, OP_ENCODE, NULL, offset, count, NULL, 0, &result);
    drop_refs(e, &s);
}

void rsj_decode_missing(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, rsj_obj present,
                        int32_t offset, int32_t count) {
    arrays s;
    if (take_shards(e, b, c, shards, &s)) return;
    /* checkBuffersAndSizes first (ReedSolomon.java:185), then shardPresent[i]
     * for i < totalShardCount (:190-194) */
    int rc = b->check_buffers_and_sizes(c, s.n, s.len, offset, count);
    if (rc) {
        throw_rc(e, b, rc);
        drop_refs(e, &s);
        return;
    }
    if (!present) {
        e->throw_new(e, NPE, "shardPresent is null");
        drop_refs(e, &s);
        return;
    }
    const int np = e->array_length(e, present);
    if (np < s.n) {
        throw_index(e, np, np);
        drop_refs(e, &s);
        return;
    }
    uint8_t pres[RSJ_MAX_SHARDS];
    e->bool_region_get(e, present, 0, s.n, pres);
    if (e->exception_pending(e)) {
        drop_refs(e, &s);
        return;
    }
    int role[RSJ_MAX_SHARDS];
    for (int i = 0; i < s.n; i++) role[i] = pres[i] ? ROLE_IN : ROLE_OUT;
    int result;
    shard_call(e, b, c, &s, role, OP_DECODE, pres, offset, count, NULL, 0, &result);
    drop_refs(e, &s);
}

int rsj_is_parity_correct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, int32_t first,
                          int32_t count, rsj_obj temp) {
    arrays s;
    if (take_shards(e, b, c, shards, &s)) return 0;
    int role[RSJ_MAX_SHARDS];
    for (int i = 0; i < s.n; i++) role[i] = ROLE_IN;
    /* the GPU needs no scratch: only tempBuffer's length is checked (ReedSolomon.java:150) */
    static const uint8_t dummy = 0;
    const int64_t temp_len = temp ? e->array_length(e, temp) : 0;
    int result = 0;
    const int rc = shard_call(e, b, c, &s, role, OP_VERIFY, NULL, first, count, temp ? &dummy : NULL, temp_len,
                              &result);
    drop_refs(e, &s);
    return rc ? 0 : result;
}

/* ---- CodingLoop natives ---- */

/* matrixRows[0..nrows) as C rows of ncols bytes.  Java reads
 * matrixRows[o][i] for i < inputCount: a null row is a NullPointerException,
 * a short one an ArrayIndexOutOfBoundsException. */
static int take_rows(rsj_env *e, rsj_obj rows, int nrows, int ncols, uint8_t *flat, const uint8_t **ptrs) {
    if (!rows) {
        e->throw_new(e, NPE, "matrixRows is null");
        return -1;
    }
    const int have = e->array_length(e, rows);
    if (have < nrows) {
        throw_index(e, have, have);
        return -1;
    }
    for (int r = 0; r < nrows; r++) {
        rsj_obj a = e->object_element(e, rows, r);
        if (e->exception_pending(e)) return -1;
        if (!a) {
            e->throw_new(e, NPE, "matrix row is null");
            return -1;
        }
        const int len = e->array_length(e, a);
        if (len < ncols) {
            e->delete_local(e, a);
            throw_index(e, len, len);
            return -1;
        }
        e->byte_region_get(e, a, 0, ncols, flat + (size_t)r * ncols);
        e->delete_local(e, a);
        if (e->exception_pending(e)) return -1;
        ptrs[r] = flat + (size_t)r * ncols;
    }
    return 0;
}

/* inputs[0..nin) and outputs[0..nout): counts against the array lengths,
 * then every array must hold [offset, offset + count) (the Java loops index
 * each of them over that range). */
static int take_io(rsj_env *e, rsj_obj ins, int nin, rsj_obj outs, int nout, int32_t offset, int32_t count,
                   arrays *in, arrays *out) {
    in->n = out->n = 0;
    if (!ins || !outs) {
        e->throw_new(e, NPE, ins ? "outputs is null" : "inputs is null");
        return -1;
    }
    const int li = e->array_length(e, ins), lo = e->array_length(e, outs);
    if (nin > li) {
        throw_index(e, li, li);
        return -1;
    }
    if (nout > lo) {
        throw_index(e, lo, lo);
        return -1;
    }
    if (take(e, ins, nin, in)) return -1;
    if (take(e, outs, nout, out)) {
        drop_refs(e, in);
        return -1;
    }
    if (count > 0) {
        arrays *all[2] = {in, out};
        for (int w = 0; w < 2; w++)
            for (int i = 0; i < all[w]->n; i++) {
                const int64_t len = all[w]->len[i];
                if (offset < 0 || (int64_t)offset + count > len) {
                    throw_index(e, offset < 0 ? offset : (len > offset ? len : offset), len);
                    drop_refs(e, out);
                    drop_refs(e, in);
                    return -1;
                }
            }
    }
    return 0;
}

static int loop_call(rsj_env *e, const rsj_backend *b, rsj_obj rows, rsj_obj ins, int32_t nin, rsj_obj outs,
                     int32_t nout, int32_t offset, int32_t count, int verify) {
    if (nin < 0 || nout < 0 || nin > RSJ_MAX_SHARDS || nout > RSJ_MAX_SHARDS) {
        e->throw_new(e, IAE, "input/output count out of range (0..256)");
        return -1;
    }
    int result = 1;
    if (nout == 0) return 1;
    uint8_t *flat = (uint8_t *)malloc((size_t)nout * (nin > 0 ? nin : 1));
    const uint8_t *rp[RSJ_MAX_SHARDS];
    if (!flat) {
        e->throw_new(e, "java/lang/OutOfMemoryError", "matrix rows");
        return -1;
    }
    if (take_rows(e, rows, nout, nin, flat, rp)) {
        free(flat);
        return -1;
    }
    arrays in, out;
    if (take_io(e, ins, nin, outs, nout, offset, count, &in, &out)) {
        free(flat);
        return -1;
    }
    int rc = 0;
    /* nothing is coded when count <= 0 or nin == 0 (the Java loops do no byte iterations) */
    if (nin > 0 && count > 0) {
        movable mv;
        mv_init(&mv, e);
        for (int i = 0; i < nin; i++) mv_add(&mv, in.arr[i], in.len[i], RSJ_ABORT);
        for (int i = 0; i < nout; i++) mv_add(&mv, out.arr[i], out.len[i], verify ? RSJ_ABORT : RSJ_COMMIT);
        int copies = 0;
        rc = mv_probe(&mv, &copies);
        if (!rc && !copies) {
            const rs_relocator r = mv_relocator(&mv);
            b->set_relocator(&r);
            int part = 1;
            const uint8_t *const *ik = mv.key, *const *ok = mv.key + nin;
            const int brc = verify ? b->check_some_shards(rp, ik, nin, ok, nout, offset, count, &part)
                                   : b->code_some_shards(rp, ik, nin, (uint8_t *const *)ok, nout, offset, count);
            b->set_relocator(NULL);
            rc = mv_result(e, b, &mv, brc);
            if (!rc && !part) result = 0;
        } else if (!rc) {  /* the JVM copies: slices through C buffers */
            uint8_t *ib[RSJ_MAX_SHARDS], *ob[RSJ_MAX_SHARDS];
            uint8_t *mi = slice_buffers(nin, ib), *mo = slice_buffers(nout, ob);
            if (!mi || !mo) {
                e->throw_new(e, "java/lang/OutOfMemoryError", "slice buffers");
                rc = -1;
            }
            for (int32_t done = 0; !rc && done < count && result;) {
                const int32_t n = (count - done) < (int32_t)RSJ_SLICE_BYTES ? (count - done) : (int32_t)RSJ_SLICE_BYTES;
                int part = 1;
                for (int i = 0; i < nin; i++) e->byte_region_get(e, in.arr[i], offset + done, n, ib[i]);
                if (verify)
                    for (int i = 0; i < nout; i++) e->byte_region_get(e, out.arr[i], offset + done, n, ob[i]);
                if (e->exception_pending(e)) {
                    rc = -1;
                    break;
                }
                const int brc = verify ? b->check_some_shards(rp, (const uint8_t *const *)ib, nin,
                                                              (const uint8_t *const *)ob, nout, 0, n, &part)
                                       : b->code_some_shards(rp, (const uint8_t *const *)ib, nin, ob, nout, 0, n);
                if (brc) {
                    throw_rc(e, b, brc);
                    rc = -1;
                    break;
                }
                if (!verify)
                    for (int i = 0; i < nout; i++) e->byte_region_set(e, out.arr[i], offset + done, n, ob[i]);
                if (e->exception_pending(e)) {
                    rc = -1;
                    break;
                }
                if (!part) result = 0;
                done += n;
            }
            free(mi);
            free(mo);
        }
    }
    drop_refs(e, &out);
    drop_refs(e, &in);
    free(flat);
    return rc ? -1 : result;
}

void rsj_code_some_shards(rsj_env *e, const rsj_backend *b, rsj_obj rows, rsj_obj inputs, int32_t nin,
                          rsj_obj outputs, int32_t nout, int32_t offset, int32_t count) {
    (void)loop_call(e, b, rows, inputs, nin, outputs, nout, offset, count, 0);
}

int rsj_check_some_shards(rsj_env *e, const rsj_backend *b, rsj_obj rows, rsj_obj inputs, int32_t nin,
                          rsj_obj to_check, int32_t ncheck, int32_t offset, int32_t count) {
    const int r = loop_call(e, b, rows, inputs, nin, to_check, ncheck, offset, count, 1);
    return r > 0;
}

void rsj_recover_groups_shard_major(rsj_env *e, const rsj_backend *b, const rs_codec *c, int64_t dev_base,
                                    int64_t server_stride, int32_t chunk_len, int64_t n_groups, rsj_obj present,
                                    int64_t stream) {
    if (!present) {
        e->throw_new(e, NPE, "present is null");
        return;
    }
    if (server_stride < 0 || chunk_len < 0 || n_groups < 0) {
        e->throw_new(e, IAE, "negative size");
        return;
    }
    const int total = b->total_shards(c);
    const int n = e->array_length(e, present);
    if (total <= 0 || n_groups > INT32_MAX / total || (int64_t)n != n_groups * total) {
        char msg[128];
        snprintf(msg, sizeof msg, "present has %d flags; n_groups * total shards is %lld", n,
                 (long long)n_groups * (total > 0 ? total : 0));
        e->throw_new(e, IAE, msg);
        return;
    }
    /* Copied out (GetByteArrayRegion), not pinned: the call can block (plan
     * uploads, waits on the previous call's event), and a critical region
     * held that long stalls the GC.  The library reads the flags on the host
     * only. */
    uint8_t *flags = n ? (uint8_t *)malloc((size_t)n) : NULL;
    if (n && !flags) {
        e->throw_new(e, "java/lang/OutOfMemoryError", "present flags");
        return;
    }
    if (n) {
        e->byte_region_get(e, present, 0, n, flags);
        if (e->exception_pending(e)) {
            free(flags);
            return;
        }
    }
    static const uint8_t none = 0;
    const int rc = b->decode_groups_shard_major(c, (uint8_t *)(uintptr_t)dev_base, (size_t)server_stride,
                                                (size_t)chunk_len, (size_t)n_groups, flags ? flags : &none,
                                                (void *)(uintptr_t)stream);
    free(flags);
    if (rc) throw_rc(e, b, rc);
}

/* present (byte[] of n_groups * total flags) copied out, validated; NULL
 * with an exception pending on failure (the caller frees the result). */
static uint8_t *take_group_flags(rsj_env *e, rsj_obj present, int total, int64_t n_groups, int *nflags) {
    static uint8_t none;
    if (!present) {
        e->throw_new(e, NPE, "present is null");
        return NULL;
    }
    const int n = e->array_length(e, present);
    if (total <= 0 || n_groups < 0 || n_groups > INT32_MAX / total || (int64_t)n != n_groups * total) {
        char msg[128];
        snprintf(msg, sizeof msg, "present has %d flags; nGroups * total shards is %lld", n,
                 (long long)n_groups * (total > 0 ? total : 0));
        e->throw_new(e, IAE, msg);
        return NULL;
    }
    *nflags = n;
    if (!n) return &none;
    uint8_t *flags = (uint8_t *)malloc((size_t)n);
    if (!flags) {
        e->throw_new(e, "java/lang/OutOfMemoryError", "present flags");
        return NULL;
    }
    e->byte_region_get(e, present, 0, n, flags);
    if (e->exception_pending(e)) {
        free(flags);
        return NULL;
    }
    return flags;
}

void rsj_recover_groups_shard_major_host(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj servers,
                                         int32_t chunk_len, int32_t n_groups, rsj_obj present) {
    arrays s;
    if (take_shards(e, b, c, servers, &s)) return;
    if (chunk_len < 0 || n_groups < 0) {
        e->throw_new(e, IAE, "negative size");
        drop_refs(e, &s);
        return;
    }
    int nflags = 0;
    uint8_t *flags = take_group_flags(e, present, s.n, n_groups, &nflags);
    if (!flags) {
        drop_refs(e, &s);
        return;
    }
    /* every server array is read (its present chunks) and written (its absent ones) */
    movable mv;
    mv_init(&mv, e);
    for (int i = 0; i < s.n; i++) mv_add(&mv, s.arr[i], s.len[i], RSJ_COMMIT);
    int copies = 0;
    if (!mv_probe(&mv, &copies)) {
        if (copies) {
            /* the JVM copies: the whole call through C buffers (the master's
             * arrays are one chunk per group per server: a few MB at most) */
            const int64_t span = (int64_t)chunk_len * n_groups;
            uint8_t *buf[RSJ_MAX_SHARDS];
            uint8_t *mem = span > 0 ? (uint8_t *)malloc((size_t)(span * s.n)) : NULL;
            int64_t lens[RSJ_MAX_SHARDS];
            if (span > 0 && !mem) {
                e->throw_new(e, "java/lang/OutOfMemoryError", "group buffers");
            } else {
                for (int i = 0; i < s.n; i++) {
                    buf[i] = mem ? mem + (size_t)(span * i) : NULL;
                    lens[i] = span;
                    if (span > s.len[i]) {
                        throw_index(e, s.len[i], s.len[i]);
                        break;
                    }
                    if (span) e->byte_region_get(e, s.arr[i], 0, (int)span, buf[i]);
                }
                const int rc = e->exception_pending(e) ? 0
                               : b->decode_groups_shard_major_host(c, buf, s.n, lens, (size_t)chunk_len,
                                                                    (size_t)n_groups, flags);
                if (rc) throw_rc(e, b, rc);
                for (int i = 0; !e->exception_pending(e) && span && i < s.n; i++)
                    e->byte_region_set(e, s.arr[i], 0, (int)span, buf[i]);
            }
            free(mem);
        } else {
            const rs_relocator r = mv_relocator(&mv);
            b->set_relocator(&r);
            const int rc = b->decode_groups_shard_major_host(c, (uint8_t *const *)mv.key, s.n, s.len,
                                                             (size_t)chunk_len, (size_t)n_groups, flags);
            b->set_relocator(NULL);
            (void)mv_result(e, b, &mv, rc);
        }
    }
    if (nflags) free(flags);
    drop_refs(e, &s);
}

/* ---- client file layout natives (ReedSolomonEncoder / ReedSolomonDecoder) ---- */

typedef struct {
    int op;                 /* OP_ENCODE or OP_DECODE */
    int32_t block;
    int64_t file_len;       /* encode: the file's length; decode: fileSize */
    int32_t byte_cnt;       /* decode, whole call: byteCntInShard */
    const uint8_t *present; /* decode */
} file_op;

/* The whole call: the arrays as Java holds them, every argument passed on, so
 * the library makes every check itself. */
static int file_whole(const rsj_backend *b, const rs_codec *c, const file_op *op, uint8_t *const *sh, int n,
                      const int64_t *len, uint8_t *f) {
    if (op->op == OP_ENCODE) return b->file_encode(c, f, op->file_len, op->block, sh, n, len);
    return b->file_decode(c, sh, n, len, op->present, op->byte_cnt, op->block, f, op->file_len);
}

/* Block rows [r0, r1) of a sliced call: row r0 of every shard at sh[i], the
 * file's row r0 at f (only the file's own bytes in those rows are read or
 * written; NULL when the rows hold none). */
static int file_rows(const rsj_backend *b, const rs_codec *c, const file_op *op, uint8_t *const *sh, int n,
                     uint8_t *f, int64_t r0, int64_t r1) {
    const int64_t kb = (int64_t)b->data_shards(c) * op->block, len = (r1 - r0) * op->block;
    int64_t fl = op->file_len - r0 * kb;
    if (fl < 0) fl = 0;
    if (fl > (r1 - r0) * kb) fl = (r1 - r0) * kb;
    int64_t lens[RSJ_MAX_SHARDS];
    for (int i = 0; i < n; i++) lens[i] = len;
    if (op->op == OP_ENCODE) return b->file_encode(c, fl ? f : NULL, fl, op->block, sh, n, lens);
    return b->file_decode(c, sh, n, lens, op->present, (int32_t)len, op->block, fl ? f : NULL, fl);
}

static int64_t slice_rows(int32_t block) {
    const int64_t per = (int64_t)RSJ_SLICE_BYTES / block;
    return per > 0 ? per : 1;
}

/* Runs a file call over the shard arrays s (roles: what each is) and the file
 * array f (f_role: read for encode, written for decode): one library call
 * with every array movable (the file header); when the JVM copies and the
 * rows exceed one slice, slice by slice through C buffers (validated up
 * front by the callers).  Leaves an exception pending on failure. */
static void file_call(rsj_env *e, const rsj_backend *b, const rs_codec *c, const file_op *op, arrays *s,
                      const int *role, rsj_obj f, int f_role, int64_t rows) {
    const int64_t blk = op->block, kb = (int64_t)b->data_shards(c) * blk, per = slice_rows(op->block);
    const int64_t f_len = e->array_length(e, f);
    movable mv;
    mv_init(&mv, e);
    for (int i = 0; i < s->n; i++) mv_add(&mv, s->arr[i], s->len[i], (role[i] & ROLE_OUT) ? RSJ_COMMIT : RSJ_ABORT);
    mv_add(&mv, f, f_len, f_role == ROLE_OUT ? RSJ_COMMIT : RSJ_ABORT);
    int copies = 0;
    if (mv_probe(&mv, &copies)) return;
    if (!copies || rows <= per) {
        const rs_relocator r = mv_relocator(&mv);
        b->set_relocator(&r);
        const int rc = file_whole(b, c, op, (uint8_t *const *)mv.key, s->n, s->len, (uint8_t *)mv.key[s->n]);
        b->set_relocator(NULL);
        (void)mv_result(e, b, &mv, rc);
        return;
    }
    /* the JVM copies: slices of whole block rows through C buffers */
    uint8_t *mem = (uint8_t *)malloc((size_t)(s->n * per * blk + per * kb));
    if (!mem) {
        e->throw_new(e, "java/lang/OutOfMemoryError", "slice buffers");
        return;
    }
    uint8_t *buf[RSJ_MAX_SHARDS], *fbuf = mem + (size_t)(s->n * per * blk);
    for (int i = 0; i < s->n; i++) buf[i] = mem + (size_t)(i * per * blk);
    for (int64_t r0 = 0; r0 < rows;) {
        const int64_t r1 = r0 + per < rows ? r0 + per : rows;
        const int32_t len = (int32_t)((r1 - r0) * blk);
        int64_t fl = op->file_len - r0 * kb;
        if (fl < 0) fl = 0;
        if (fl > (r1 - r0) * kb) fl = (r1 - r0) * kb;
        for (int i = 0; i < s->n; i++)
            if (role[i] & ROLE_IN) e->byte_region_get(e, s->arr[i], (int)(r0 * blk), len, buf[i]);
        if (f_role == ROLE_IN && fl) e->byte_region_get(e, f, (int)(r0 * kb), (int)fl, fbuf);
        if (e->exception_pending(e)) break;
        const int rc = file_rows(b, c, op, buf, s->n, fbuf, r0, r1);
        if (rc) {
            throw_rc(e, b, rc);
            break;
        }
        for (int i = 0; i < s->n; i++)
            if (role[i] & ROLE_OUT) e->byte_region_set(e, s->arr[i], (int)(r0 * blk), len, buf[i]);
        if (f_role == ROLE_OUT && fl) e->byte_region_set(e, f, (int)(r0 * kb), (int)fl, fbuf);
        if (e->exception_pending(e)) break;
        r0 = r1;
    }
    free(mem);
}

void rsj_file_encode(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj file, int32_t block, rsj_obj shards) {
    if (!file) {
        e->throw_new(e, NPE, "fileData is null");
        return;
    }
    arrays s;
    if (take_shards(e, b, c, shards, &s)) return;
    const int64_t flen = e->array_length(e, file);
    int64_t padded = 0, S = 0;
    int rc = b->file_layout(c, flen, block, &padded, &S);
    if (rc) {
        throw_rc(e, b, rc);
        drop_refs(e, &s);
        return;
    }
    /* checked up front (a sliced call hands the library slices only): every
     * shard holds the padded length / k, as the reference allocates them
     * (ReedSolomonEncoder.java:63) */
    for (int i = 0; i < s.n; i++)
        if (s.len[i] < S) {
            char msg[96];
            snprintf(msg, sizeof msg, "shard %d is shorter than %lld", i, (long long)S);
            e->throw_new(e, IAE, msg);
            drop_refs(e, &s);
            return;
        }
    int role[RSJ_MAX_SHARDS];
    for (int i = 0; i < s.n; i++) role[i] = ROLE_OUT; /* data shards from the file, parity coded */
    const file_op op = {OP_ENCODE, block, flen, 0, NULL};
    file_call(e, b, c, &op, &s, role, file, ROLE_IN, S / block);
    drop_refs(e, &s);
}

void rsj_file_decode(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, rsj_obj present,
                     int32_t byte_cnt, int32_t block, rsj_obj file_out, int32_t file_size) {
    arrays s;
    if (take_shards(e, b, c, shards, &s)) return;
    /* decodeMissing's checks first (ReedSolomonDecoder.java:36 -> ReedSolomon.java:185-194) */
    int rc = b->check_buffers_and_sizes(c, s.n, s.len, 0, byte_cnt);
    if (rc) {
        throw_rc(e, b, rc);
        drop_refs(e, &s);
        return;
    }
    if (!present || !file_out) {
        e->throw_new(e, NPE, present ? "fileOut is null" : "shardPresent is null");
        drop_refs(e, &s);
        return;
    }
    const int np = e->array_length(e, present);
    if (np < s.n) {
        throw_index(e, np, np);
        drop_refs(e, &s);
        return;
    }
    uint8_t pres[RSJ_MAX_SHARDS];
    e->bool_region_get(e, present, 0, s.n, pres);
    if (e->exception_pending(e)) {
        drop_refs(e, &s);
        return;
    }
    const int fo_len = e->array_length(e, file_out);
    if (file_size > fo_len) { /* the trimmed copy would run past fileOut (ReedSolomonDecoder.java:63-64) */
        throw_index(e, fo_len, fo_len);
        drop_refs(e, &s);
        return;
    }
    int role[RSJ_MAX_SHARDS], n_present = 0;
    for (int i = 0; i < s.n; i++) {
        role[i] = pres[i] ? ROLE_IN : ROLE_OUT;
        n_present += pres[i] ? 1 : 0;
    }
    /* sliced only when every slice is a valid call on its own: whole shards
     * decoded, whole block rows, enough survivors and a file that fits;
     * anything else goes to the library whole, which reports it */
    const int64_t L = s.n ? s.len[0] : 0, k = b->data_shards(c);
    const int sliceable = block >= 1 && byte_cnt == L && L % block == 0 && n_present >= k && file_size >= 0 &&
                          (int64_t)file_size <= k * L;
    const file_op op = {OP_DECODE, block, file_size, byte_cnt, pres};
    file_call(e, b, c, &op, &s, role, file_out, ROLE_OUT, sliceable ? L / block : 0);
    drop_refs(e, &s);
}

/* ---- direct ByteBuffers ---- */

rsj_obj rsj_alloc_pinned(rsj_env *e, const rsj_backend *b, int32_t capacity) {
    if (capacity < 0) {
        e->throw_new(e, IAE, "capacity is negative");
        return NULL;
    }
    void *p = NULL;
    const int rc = b->host_alloc(&p, (size_t)capacity);
    if (rc) {
        if (rc == RS_E_HIP) e->throw_new(e, "java/lang/OutOfMemoryError", b->last_error());
        else throw_rc(e, b, rc);
        return NULL;
    }
    rsj_obj buf = e->new_direct(e, p, capacity);
    if (!buf) b->host_free(p); /* NewDirectByteBuffer threw */
    return buf;
}

void rsj_free_pinned(rsj_env *e, const rsj_backend *b, rsj_obj buf) {
    if (!buf) return;
    uint8_t *p = e->direct_address(e, buf);
    if (!p) {
        e->throw_new(e, IAE, "not a direct buffer");
        return;
    }
    const int rc = b->host_free(p);
    if (rc) throw_rc(e, b, rc);
}

/* The first n elements of a ByteBuffer[] by address and capacity (local
 * references dropped as soon as the address is read: a direct buffer's
 * memory does not move). */
static int take_direct(rsj_env *e, rsj_obj outer, int n, uint8_t **ptr, int64_t *len) {
    if (n > RSJ_MAX_SHARDS) n = RSJ_MAX_SHARDS;
    for (int i = 0; i < n; i++) {
        rsj_obj x = e->object_element(e, outer, i);
        if (e->exception_pending(e)) return -1;
        if (!x) {
            e->throw_new(e, NPE, "ByteBuffer element is null");
            return -1;
        }
        ptr[i] = e->direct_address(e, x);
        len[i] = ptr[i] ? e->direct_capacity(e, x) : 0;
        e->delete_local(e, x);
        if (!ptr[i]) {
            char msg[64];
            snprintf(msg, sizeof msg, "shard %d is not a direct buffer", i);
            e->throw_new(e, IAE, msg);
            return -1;
        }
    }
    return 0;
}

/* shards.length != totalShardCount first (ReedSolomon.java:280-282), then the elements. */
static int take_direct_shards(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, uint8_t **ptr,
                              int64_t *len, int *n) {
    if (!shards) {
        e->throw_new(e, NPE, "shards is null");
        return -1;
    }
    *n = e->array_length(e, shards);
    if (*n != b->total_shards(c)) {
        int64_t none = 0;
        throw_rc(e, b, b->check_buffers_and_sizes(c, *n, &none, 0, 0));
        return -1;
    }
    return take_direct(e, shards, *n, ptr, len);
}

static int take_present(rsj_env *e, rsj_obj present, int n, uint8_t *pres) {
    if (!present) {
        e->throw_new(e, NPE, "shardPresent is null");
        return -1;
    }
    const int np = e->array_length(e, present);
    if (np < n) {
        throw_index(e, np, np);
        return -1;
    }
    e->bool_region_get(e, present, 0, n, pres);
    return e->exception_pending(e) ? -1 : 0;
}

void rsj_encode_parity_direct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, int32_t offset,
                              int32_t count) {
    uint8_t *ptr[RSJ_MAX_SHARDS];
    int64_t len[RSJ_MAX_SHARDS];
    int n = 0;
    if (take_direct_shards(e, b, c, shards, ptr, len, &n)) return;
    const int rc = b->encode_parity(c, ptr, n, len, offset, count);
    if (rc) throw_rc(e, b, rc);
}

void rsj_decode_missing_direct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, rsj_obj present,
                               int32_t offset, int32_t count) {
    uint8_t *ptr[RSJ_MAX_SHARDS], pres[RSJ_MAX_SHARDS];
    int64_t len[RSJ_MAX_SHARDS];
    int n = 0;
    if (take_direct_shards(e, b, c, shards, ptr, len, &n)) return;
    /* checkBuffersAndSizes first (ReedSolomon.java:185), then shardPresent[i] (:190-194) */
    int rc = b->check_buffers_and_sizes(c, n, len, offset, count);
    if (rc) {
        throw_rc(e, b, rc);
        return;
    }
    if (take_present(e, present, n, pres)) return;
    rc = b->decode_missing(c, ptr, n, len, pres, offset, count);
    if (rc) throw_rc(e, b, rc);
}

void rsj_file_encode_direct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj file, int32_t file_len,
                            int32_t block, rsj_obj shards) {
    if (!file) {
        e->throw_new(e, NPE, "fileData is null");
        return;
    }
    uint8_t *f = e->direct_address(e, file);
    if (!f) {
        e->throw_new(e, IAE, "fileData is not a direct buffer");
        return;
    }
    if (file_len > e->direct_capacity(e, file)) {
        const int64_t cap = e->direct_capacity(e, file);
        throw_index(e, cap, cap);
        return;
    }
    uint8_t *ptr[RSJ_MAX_SHARDS];
    int64_t len[RSJ_MAX_SHARDS];
    int n = 0;
    if (take_direct_shards(e, b, c, shards, ptr, len, &n)) return;
    const int rc = b->file_encode(c, f, file_len, block, ptr, n, len);
    if (rc) throw_rc(e, b, rc);
}

void rsj_file_decode_direct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj shards, rsj_obj present,
                            int32_t byte_cnt, int32_t block, rsj_obj file_out, int32_t file_size) {
    uint8_t *ptr[RSJ_MAX_SHARDS], pres[RSJ_MAX_SHARDS];
    int64_t len[RSJ_MAX_SHARDS];
    int n = 0;
    if (take_direct_shards(e, b, c, shards, ptr, len, &n)) return;
    int rc = b->check_buffers_and_sizes(c, n, len, 0, byte_cnt);
    if (rc) {
        throw_rc(e, b, rc);
        return;
    }
    if (take_present(e, present, n, pres)) return;
    if (!file_out) {
        e->throw_new(e, NPE, "fileOut is null");
        return;
    }
    uint8_t *f = e->direct_address(e, file_out);
    if (!f) {
        e->throw_new(e, IAE, "fileOut is not a direct buffer");
        return;
    }
    const int64_t cap = e->direct_capacity(e, file_out);
    if (file_size > cap) {
        throw_index(e, cap, cap);
        return;
    }
    rc = b->file_decode(c, ptr, n, len, pres, byte_cnt, block, f, file_size);
    if (rc) throw_rc(e, b, rc);
}

void rsj_recover_groups_shard_major_direct(rsj_env *e, const rsj_backend *b, const rs_codec *c, rsj_obj servers,
                                           int32_t chunk_len, int32_t n_groups, rsj_obj present) {
    uint8_t *ptr[RSJ_MAX_SHARDS];
    int64_t len[RSJ_MAX_SHARDS];
    int n = 0;
    if (take_direct_shards(e, b, c, servers, ptr, len, &n)) return;
    if (chunk_len < 0 || n_groups < 0) {
        e->throw_new(e, IAE, "negative size");
        return;
    }
    int nflags = 0;
    uint8_t *flags = take_group_flags(e, present, n, n_groups, &nflags);
    if (!flags) return;
    const int rc = b->decode_groups_shard_major_host(c, ptr, n, len, (size_t)chunk_len, (size_t)n_groups, flags);
    if (nflags) free(flags);
    if (rc) throw_rc(e, b, rc);
}
