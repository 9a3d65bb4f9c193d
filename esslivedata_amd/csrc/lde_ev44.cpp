// lde_ev44.cpp -- in-place decoder of ev44 flatbuffer messages (host side of
// the boundary; no HIP).
//
// Replaces the per-message decode the reference runs in Python through
// ess-streaming-data-types 0.27.0 / flatbuffers 25.12.19
// (requirements/base.txt):
//   KafkaToEv44Adapter.adapt           SRC/kafka/message_adapter.py:192-204
//   KafkaToMonitorEventsAdapter.adapt  SRC/kafka/message_adapter.py:356-409
// Neither library is vendored under /root/reference, so the wire format is
// restated from their published definitions:
//
//   file_identifier "ev44";
//   table Event44Message {
//     source_name : string;            // field 0
//     message_id : long;               // field 1 (default 0)
//     reference_time : [long];         // field 2 (pulse times, ns since epoch)
//     reference_time_index : [int];    // field 3
//     time_of_flight : [int];          // field 4 (ns)
//     pixel_id : [int];                // field 5
//   }
//
// Flatbuffer layout rules used here: bytes [0,4) hold the little-endian
// uoffset of the root table, [4,8) the file identifier; a table starts with
// an soffset to its vtable (vtable = table - soffset); the vtable is
// u16 vtable_size, u16 table_size, then one u16 offset per field (0 or beyond
// vtable_size = absent); strings and vectors are reached through a uoffset
// stored in the table (target = field position + value) and start with a u32
// element count.
//
// Unlike the Python accessors, every offset, count and extent is checked
// against the buffer, so hostile payloads (tests/helpers/hostile_wire.py in
// the reference: garbage, empty, truncated, wrong schema) fail with an error
// instead of reading out of bounds.  Vectors are returned as pointers into
// the caller's buffer (zero copy, like the reference's *AsNumpy views); they
// may be unaligned, so consumers copy them with memcpy.

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/lde.h"
#include "lde_internal.h"

namespace {

inline uint32_t rd_u32(const uint8_t *p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
inline int32_t rd_i32(const uint8_t *p) {
    int32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
inline uint16_t rd_u16(const uint8_t *p) {
    uint16_t v;
    std::memcpy(&v, p, 2);
    return v;
}

struct Reader {
    const uint8_t *b;
    int64_t n;
    int64_t table = 0, vt = 0;
    int vt_size = 0, tbl_size = 0;
    std::string *err;

    int bad(const char *what) {
        if (err) *err = std::string("ev44: ") + what;
        return LDE_EINVAL;
    }
    bool in(int64_t pos, int64_t len) const { return pos >= 0 && len >= 0 && pos <= n && len <= n - pos; }

    // offset of field i inside the table, 0 when absent; -1 when malformed
    int64_t field(int i, int size) {
        const int slot = 4 + 2 * i;
        if (slot + 2 > vt_size) return 0;
        const int off = rd_u16(b + vt + slot);
        if (off == 0) return 0;
        if (off < 4 || off + size > tbl_size) return -1;
        return off;
    }

    // uoffset field -> (target position, element count); rc != 0 on error
    int ref(int i, int64_t elem, const char *name, const uint8_t **data, int64_t *count, bool *present) {
        *present = false;
        *data = nullptr;
        *count = 0;
        const int64_t off = field(i, 4);
        if (off < 0) return bad(name);
        if (off == 0) return LDE_OK;
        const int64_t pos = table + off;
        const int64_t tgt = pos + (int64_t)rd_u32(b + pos);
        if (!in(tgt, 4)) return bad(name);
        const int64_t cnt = rd_u32(b + tgt);
        if (!in(tgt + 4, cnt * elem)) return bad(name);
        *data = b + tgt + 4;
        *count = cnt;
        *present = true;
        return LDE_OK;
    }
};

}  // namespace

namespace lde {

int ev44_parse(const uint8_t *buf, int64_t len, lde_ev44_view *v, std::string *err) {
    if (!v) {
        if (err) *err = "ev44: view is NULL";
        return LDE_EINVAL;
    }
    std::memset(v, 0, sizeof(*v));
    Reader r{buf, len};
    r.err = err;
    if (len < 0 || (!buf && len > 0)) return r.bad("buffer is NULL");
    if (len < 8) return r.bad("buffer too short for a flatbuffer");
    if (std::memcmp(buf + 4, "ev44", 4) != 0) {
        char got[5];
        for (int i = 0; i < 4; ++i) got[i] = (buf[4 + i] >= 32 && buf[4 + i] < 127) ? (char)buf[4 + i] : '?';
        got[4] = 0;
        if (err) *err = std::string("ev44: wrong schema identifier '") + got + "', expected 'ev44'";
        return LDE_EINVAL;
    }
    r.table = rd_u32(buf);
    if (!r.in(r.table, 4)) return r.bad("root table offset out of range");
    r.vt = r.table - (int64_t)rd_i32(buf + r.table);
    if (!r.in(r.vt, 4)) return r.bad("vtable offset out of range");
    r.vt_size = rd_u16(buf + r.vt);
    r.tbl_size = rd_u16(buf + r.vt + 2);
    if (r.vt_size < 4 || (r.vt_size & 1) || !r.in(r.vt, r.vt_size)) return r.bad("malformed vtable");
    if (r.tbl_size < 4 || !r.in(r.table, r.tbl_size)) return r.bad("table extends past the buffer");

    const uint8_t *p;
    int64_t cnt;
    bool present;
    int rc;
    if ((rc = r.ref(0, 1, "source_name out of range", &p, &cnt, &present))) return rc;
    if (present) {
        v->source_name = (const char *)p;
        v->source_name_len = cnt;
        v->present |= LDE_EV44_HAS_SOURCE_NAME;
    }
    const int64_t mid = r.field(1, 8);
    if (mid < 0) return r.bad("message_id out of range");
    if (mid > 0) {
        std::memcpy(&v->message_id, buf + r.table + mid, 8);
        v->present |= LDE_EV44_HAS_MESSAGE_ID;
    }
    struct {
        int field;
        int64_t elem;
        const char *what;
        const void **data;
        int64_t *count;
        uint32_t bit;
    } vecs[] = {
        {2, 8, "reference_time out of range", &v->reference_time, &v->n_reference_time,
         LDE_EV44_HAS_REFERENCE_TIME},
        {3, 4, "reference_time_index out of range", &v->reference_time_index,
         &v->n_reference_time_index, LDE_EV44_HAS_REFERENCE_TIME_INDEX},
        {4, 4, "time_of_flight out of range", &v->time_of_flight, &v->n_time_of_flight,
         LDE_EV44_HAS_TIME_OF_FLIGHT},
        {5, 4, "pixel_id out of range", &v->pixel_id, &v->n_pixel_id, LDE_EV44_HAS_PIXEL_ID},
    };
    for (auto &e : vecs) {
        if ((rc = r.ref(e.field, e.elem, e.what, &p, &cnt, &present))) return rc;
        if (present) {
            *e.data = p;
            *e.count = cnt;
            v->present |= e.bit;
        }
    }
    return LDE_OK;
}

int ev44_events(const lde_ev44_view *v, int64_t kafka_timestamp_ms, int32_t flags,
                int64_t *timestamp_ns, std::string *err) {
    // timestamp: reference_time[-1], else the Kafka timestamp (ms -> ns),
    // message_adapter.py:197-201 / :393-397.  An absent reference_time vector
    // raises in the reference (the flatbuffers accessor returns a scalar 0
    // whose `.size` fails) and the message is dropped
    // (tests/kafka/adapter_robustness_test.py:98-108, strict xfail).
    if (!(v->present & LDE_EV44_HAS_REFERENCE_TIME)) {
        if (err) *err = "ev44: reference_time vector is absent";
        return LDE_EINVAL;
    }
    if (!(v->present & LDE_EV44_HAS_SOURCE_NAME)) {
        if (err) *err = "ev44: source_name is absent";
        return LDE_EINVAL;
    }
    if (!(v->present & LDE_EV44_HAS_TIME_OF_FLIGHT)) {
        if (err) *err = "ev44: time_of_flight vector is absent";
        return LDE_EINVAL;
    }
    const bool detector = (flags & LDE_EV44_MONITOR) == 0;
    if (detector && !(v->present & LDE_EV44_HAS_PIXEL_ID)) {
        if (err) *err = "ev44: pixel_id vector is absent";
        return LDE_EINVAL;
    }
    if (flags & LDE_EV44_SINGLE_PULSE) {
        // _require_single_pulse, to_nxevent_data.py:16-19 (index[0] of an
        // empty index raises IndexError in the reference: rejected here too)
        int32_t idx0 = 0;
        if (v->n_reference_time_index > 0) std::memcpy(&idx0, v->reference_time_index, 4);
        if (v->n_reference_time_index != 1 || idx0 != 0 || v->n_reference_time > 1) {
            if (err) *err = "Processing multi-pulse messages is not supported.";
            return LDE_ENOTSUP;
        }
    }
    if (detector && v->n_pixel_id != v->n_time_of_flight) {
        // DetectorEvents.__post_init__, to_nxevent_data.py:57-62
        char msg[160];
        std::snprintf(msg, sizeof msg,
                      "pixel_id and time_of_arrival must have the same length, got %lld and %lld",
                      (long long)v->n_pixel_id, (long long)v->n_time_of_flight);
        if (err) *err = msg;
        return LDE_EINVAL;
    }
    if (timestamp_ns) {
        if (v->n_reference_time > 0)
            std::memcpy(timestamp_ns, (const uint8_t *)v->reference_time + 8 * (v->n_reference_time - 1), 8);
        else
            *timestamp_ns = kafka_timestamp_ms * 1000000LL;  // Timestamp.from_ms
    }
    return LDE_OK;
}

}  // namespace lde
