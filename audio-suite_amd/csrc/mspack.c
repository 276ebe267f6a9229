/*
 * mspack.c -- the native dict -> msg_preset packer (CPython extension _mspack).
 *
 * render(params) reads its params dict (microsound_0.2.1/main_v2.py:588-792,
 * "MS") with int(...) / float(...) at each use, truthiness for the switches and
 * string matches for the modes.  msgpu.pack.pack_preset states that mapping in
 * Python; this module does the same per dict in one C pass, so a batch of 1024
 * dicts packs in about a millisecond instead of tens.
 *
 *   pack(dicts, presets, out_n, defaults, gen_modes, processes, lane_cb, src_cb)
 *
 * dicts      list of params dicts; an absent key takes defaults[key] (what
 *            msgpu.merged gives; the drop-in checks missing keys before this)
 * presets    writable buffer of len(dicts) msg_preset (include/msgpu.h)
 * out_n      writable int64 buffer of len(dicts): int(max(1, round(dur * sr)))
 * gen_modes  name -> msg_gen_mode (absent: MSG_GEN_FALLBACK, MS:686)
 * processes  name -> msg_process (absent: MSG_PROC_NONE, MS:558)
 * lane_cb    lane string -> (first pair, pairs) in the batch's breakpoint bank
 *            (msgpu.pack.Banks.lane, which parses with MS:452-467's rules);
 *            called once per distinct string object
 * src_cb     dict -> (ir_conv, F_SPACE_IR or 0, ir_frag, image)
 *            (msgpu.pack.sources); called once per distinct (IR object,
 *            space_ir_max_samps, space_ir_on, gen_mode, image object)
 *
 * Every conversion is the Python one (PyNumber_Float == float(), PyNumber_Long
 * == int(), PyObject_IsTrue == bool()), so the errors are the reference's too.
 * Test infrastructure holds it byte-identical to pack_preset
 * (tests/test_pack_native.py).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <math.h>
#include <stddef.h>
#include <string.h>

#include "../../include/msgpu.h"

enum { K_F64, K_I64, K_I32 };
typedef struct { const char* key; size_t off; int kind; } Field;

#define FD(name) {#name, offsetof(msg_preset, name), K_F64}
#define FI(name) {#name, offsetof(msg_preset, name), K_I32}
static const Field kFields[] = {
    {"seed", offsetof(msg_preset, seed), K_I64},
    FI(base_sr), FI(max_grains), FI(cluster_size), FI(crackle_kernel), FI(wav_count), FI(pl_top_n),
    FI(pl_neigh), FI(res_modes), FI(wg_lines), FI(er_taps),
    FD(out_dur_s), FD(time_unfold), FD(peak), FD(sat_drive), FD(stereo_width), FD(micro_ms),
    FD(dust_density), FD(noise_tilt), FD(ring_hz), FD(ring_decay_ms), FD(crackle_alpha),
    FD(crackle_density), FD(ss_threshold), FD(ss_build), FD(ss_decay), FD(ss_noise), FD(chaos_r),
    FD(chaos_gate), FD(wav_base_hz), FD(wav_spread), FD(partial_stretch), FD(nl_warp_power),
    FD(cep_factor), FD(mb_roll), FD(bandlimit_out_hz), FD(bandlimit_roll_hz), FD(grains_per_sec),
    FD(grain_amp_rand), FD(grain_offset_max_ms), FD(cluster_spread_ms), FD(hawkes_gain),
    FD(hawkes_decay_s), FD(res_fmin), FD(res_fmax), FD(res_decay_ms), FD(wg_max_ms), FD(wg_fb),
    FD(event_feedback_amt), FD(spectral_imprint_amt), FD(spectral_imprint_smooth), FD(er_max_ms),
    FD(env_a), FD(env_d), FD(env_s), FD(env_r), FD(env_curve),
    {"mb_b1", offsetof(msg_preset, mb_b), K_F64}, {"mb_b2", offsetof(msg_preset, mb_b) + 8, K_F64},
    {"mb_b3", offsetof(msg_preset, mb_b) + 16, K_F64}, {"mb_u1", offsetof(msg_preset, mb_u), K_F64},
    {"mb_u2", offsetof(msg_preset, mb_u) + 8, K_F64}, {"mb_u3", offsetof(msg_preset, mb_u) + 16, K_F64},
};
#define N_FIELDS ((int)(sizeof(kFields) / sizeof(kFields[0])))

static const struct { const char* key; uint32_t bit; } kFlags[] = {
    {"stereo_on", MSG_F_STEREO}, {"bandlimit_on", MSG_F_BANDLIMIT}, {"partial_lock_on", MSG_F_PARTIAL_LOCK},
    {"nl_warp_on", MSG_F_NL_WARP}, {"cep_warp_on", MSG_F_CEP_WARP}, {"grain_offset_on", MSG_F_GRAIN_OFFSET},
    {"res_bank_on", MSG_F_RES_BANK}, {"wg_on", MSG_F_WAVEGUIDE}, {"event_feedback_on", MSG_F_EVENT_FEEDBACK},
    {"spectral_imprint_on", MSG_F_IMPRINT}, {"er_cloud_on", MSG_F_ER_CLOUD},
};
#define N_FLAGS ((int)(sizeof(kFlags) / sizeof(kFlags[0])))
static const char* kLanes[4] = {"bp_density", "bp_unfold", "bp_cutoff", "bp_stretch"};   /* MS:602-605 */

static PyObject* g_field_keys[N_FIELDS];
static PyObject* g_flag_keys[N_FLAGS];
static PyObject* g_lane_keys[4];
static PyObject *g_gen_mode, *g_process, *g_unfold_mode, *g_classic, *g_ir_audio, *g_img_gray, *g_max_samps,
    *g_space_ir_on;

/* p[key], else defaults[key]; borrowed; NULL with an exception set when both lack it */
static PyObject* get(PyObject* d, PyObject* defaults, PyObject* key) {
    PyObject* v = PyDict_GetItemWithError(d, key);
    if (v || PyErr_Occurred()) return v;
    v = PyDict_GetItemWithError(defaults, key);
    if (!v && !PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, key);
    return v;
}
/* p.get(key) without defaults: borrowed, Py_None when absent */
static PyObject* get_opt(PyObject* d, PyObject* key) {
    PyObject* v = PyDict_GetItemWithError(d, key);
    return v ? v : (PyErr_Occurred() ? NULL : Py_None);
}

static int to_double(PyObject* v, double* out) {
    if (PyFloat_CheckExact(v)) { *out = PyFloat_AS_DOUBLE(v); return 0; }
    PyObject* f = PyNumber_Float(v);                  /* float(v) */
    if (!f) return -1;
    *out = PyFloat_AS_DOUBLE(f);
    Py_DECREF(f);
    return 0;
}
static int to_i64(PyObject* v, long long* out) {
    if (PyLong_CheckExact(v)) {
        int of = 0;
        *out = PyLong_AsLongLongAndOverflow(v, &of);
        if (!of) return (*out == -1 && PyErr_Occurred()) ? -1 : 0;
    }
    PyObject* i = PyNumber_Long(v);                   /* int(v) */
    if (!i) return -1;
    int of = 0;
    *out = PyLong_AsLongLongAndOverflow(i, &of);
    if (of) {   /* ctypes would wrap the value modulo 2^64; keep the low 64 bits the same way */
        unsigned long long u = PyLong_AsUnsignedLongLongMask(i);
        *out = (long long)u;
    }
    Py_DECREF(i);
    return PyErr_Occurred() ? -1 : 0;
}

typedef struct { PyObject* key; int32_t off, n; } LaneHit;
typedef struct { PyObject *ir, *img; long long samps; int on, mode; int32_t r[4]; } SrcHit;

static PyObject* pack(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *dicts, *defaults, *gen_modes, *processes, *lane_cb, *src_cb;
    Py_buffer pb = {0}, nb = {0};
    if (!PyArg_ParseTuple(args, "O!w*w*O!O!O!OO", &PyList_Type, &dicts, &pb, &nb, &PyDict_Type, &defaults,
                          &PyDict_Type, &gen_modes, &PyDict_Type, &processes, &lane_cb, &src_cb))
        return NULL;
    const Py_ssize_t n = PyList_GET_SIZE(dicts);
    PyObject* result = NULL;
    LaneHit lanes[4][16];
    int nl[4] = {0, 0, 0, 0};
    SrcHit srcs[8];
    int ns = 0;
    if (pb.len < n * (Py_ssize_t)sizeof(msg_preset) || nb.len < n * (Py_ssize_t)sizeof(int64_t)) {
        PyErr_SetString(PyExc_ValueError, "output buffers too small");
        goto done;
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* d = PyList_GET_ITEM(dicts, i);
        if (!PyDict_Check(d)) {
            PyErr_SetString(PyExc_TypeError, "params must be dicts");
            goto done;
        }
        msg_preset* s = (msg_preset*)pb.buf + i;
        memset(s, 0, sizeof(*s));
        char* base = (char*)s;
        long long sr_full = 0;
        for (int f = 0; f < N_FIELDS; ++f) {
            PyObject* v = get(d, defaults, g_field_keys[f]);
            if (!v) goto done;
            if (kFields[f].kind == K_F64) {
                if (to_double(v, (double*)(base + kFields[f].off))) goto done;
            } else {
                long long x;
                if (to_i64(v, &x)) goto done;
                if (kFields[f].kind == K_I64) *(int64_t*)(base + kFields[f].off) = (int64_t)x;
                else *(int32_t*)(base + kFields[f].off) = (int32_t)(uint32_t)(unsigned long long)x;
                if (f == 1) sr_full = x;
            }
        }
        /* modes (MS:686, MS:558, MS:720) */
        PyObject* v = get(d, defaults, g_gen_mode);
        if (!v) goto done;
        PyObject* code = PyDict_GetItemWithError(gen_modes, v);
        if (!code && PyErr_Occurred()) goto done;
        s->gen_mode = code ? (int32_t)PyLong_AsLong(code) : MSG_GEN_FALLBACK;
        v = get(d, defaults, g_process);
        if (!v) goto done;
        code = PyDict_GetItemWithError(processes, v);
        if (!code && PyErr_Occurred()) goto done;
        s->process = code ? (int32_t)PyLong_AsLong(code) : MSG_PROC_NONE;
        uint32_t flags = 0;
        for (int f = 0; f < N_FLAGS; ++f) {
            PyObject* b = get(d, defaults, g_flag_keys[f]);
            if (!b) goto done;
            const int t = PyObject_IsTrue(b);
            if (t < 0) goto done;
            if (t) flags |= kFlags[f].bit;
        }
        v = get(d, defaults, g_unfold_mode);
        if (!v) goto done;
        const int ne = PyObject_RichCompareBool(v, g_classic, Py_NE);
        if (ne < 0) goto done;
        if (ne) flags |= MSG_F_MULTIBAND;
        /* breakpoint lanes: the bank position of each distinct string object */
        for (int l = 0; l < 4; ++l) {
            PyObject* ls = get(d, defaults, g_lane_keys[l]);
            if (!ls) goto done;
            int hit = -1;
            for (int k = 0; k < nl[l]; ++k)
                if (lanes[l][k].key == ls) { hit = k; break; }
            if (hit < 0) {
                PyObject* r = PyObject_CallOneArg(lane_cb, ls);
                if (!r) goto done;
                long off = -1, cnt = -1;
                if (PyTuple_Check(r) && PyTuple_GET_SIZE(r) == 2) {
                    off = PyLong_AsLong(PyTuple_GET_ITEM(r, 0));
                    cnt = PyLong_AsLong(PyTuple_GET_ITEM(r, 1));
                }
                Py_DECREF(r);
                if (PyErr_Occurred()) goto done;
                if (off < 0 || cnt < 0) {
                    PyErr_SetString(PyExc_RuntimeError, "lane_cb must return (offset, count)");
                    goto done;
                }
                if (nl[l] < 16) {   /* the dict keeps the string alive for the batch */
                    lanes[l][nl[l]].key = ls; lanes[l][nl[l]].off = (int32_t)off; lanes[l][nl[l]].n = (int32_t)cnt;
                    ++nl[l];
                }
                s->bp_off[l] = (int32_t)off; s->n_bp[l] = (int32_t)cnt;
            } else {
                s->bp_off[l] = lanes[l][hit].off; s->n_bp[l] = lanes[l][hit].n;
            }
        }
        /* IR / image sources (MS:333-362, 772-773) */
        {
            PyObject* ir = get_opt(d, g_ir_audio);
            if (!ir) goto done;
            PyObject* img = s->gen_mode == MSG_GEN_IMAGE ? get_opt(d, g_img_gray) : Py_None;
            if (!img) goto done;
            PyObject* ms = get(d, defaults, g_max_samps);
            if (!ms) goto done;
            long long samps;
            if (to_i64(ms, &samps)) goto done;
            PyObject* on_o = get(d, defaults, g_space_ir_on);
            if (!on_o) goto done;
            const int on = PyObject_IsTrue(on_o);
            if (on < 0) goto done;
            int hit = -1;
            for (int k = 0; k < ns; ++k)
                if (srcs[k].ir == ir && srcs[k].img == img && srcs[k].samps == samps && srcs[k].on == on &&
                    srcs[k].mode == s->gen_mode) { hit = k; break; }
            int32_t r4[4];
            if (hit < 0) {
                PyObject* r = PyObject_CallOneArg(src_cb, d);
                if (!r) goto done;
                if (!PyTuple_Check(r) || PyTuple_GET_SIZE(r) != 4) {
                    Py_DECREF(r);
                    PyErr_SetString(PyExc_RuntimeError, "src_cb must return a 4-tuple");
                    goto done;
                }
                for (int k = 0; k < 4; ++k) r4[k] = (int32_t)PyLong_AsLong(PyTuple_GET_ITEM(r, k));
                Py_DECREF(r);
                if (PyErr_Occurred()) goto done;
                if (ns < 8) {
                    SrcHit* h = &srcs[ns++];
                    h->ir = ir; h->img = img; h->samps = samps; h->on = on; h->mode = s->gen_mode;
                    memcpy(h->r, r4, sizeof(r4));
                }
            } else {
                memcpy(r4, srcs[hit].r, sizeof(r4));
            }
            s->ir_conv = r4[0];
            flags |= (uint32_t)r4[1];
            s->ir_frag = r4[2];
            s->image = r4[3];
        }
        s->flags = flags;
        /* out_n = int(max(1, round(out_dur_s * base_sr))) (MS:589-591) */
        {
            const double x = s->out_dur_s * (double)sr_full;
            if (isnan(x)) { PyErr_SetString(PyExc_ValueError, "cannot convert float NaN to integer"); goto done; }
            if (isinf(x)) { PyErr_SetString(PyExc_OverflowError, "cannot convert float infinity to integer"); goto done; }
            const double r = nearbyint(x);   /* round-half-even under the default rounding mode */
            if (r >= 9.2e18) { PyErr_SetString(PyExc_OverflowError, "output length beyond int64"); goto done; }
            ((int64_t*)nb.buf)[i] = r > 1.0 ? (int64_t)r : 1;
        }
    }
    result = Py_None;
    Py_INCREF(result);
done:
    PyBuffer_Release(&pb);
    PyBuffer_Release(&nb);
    return result;
}

static PyMethodDef kMethods[] = {
    {"pack", pack, METH_VARARGS, "pack(dicts, presets, out_n, defaults, gen_modes, processes, lane_cb, src_cb)"},
    {NULL, NULL, 0, NULL}};
static struct PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_mspack", "Native params-dict packer", -1, kMethods,
                                     NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__mspack(void) {
    for (int f = 0; f < N_FIELDS; ++f)
        if (!(g_field_keys[f] = PyUnicode_InternFromString(kFields[f].key))) return NULL;
    for (int f = 0; f < N_FLAGS; ++f)
        if (!(g_flag_keys[f] = PyUnicode_InternFromString(kFlags[f].key))) return NULL;
    for (int l = 0; l < 4; ++l)
        if (!(g_lane_keys[l] = PyUnicode_InternFromString(kLanes[l]))) return NULL;
    if (!(g_gen_mode = PyUnicode_InternFromString("gen_mode")) ||
        !(g_process = PyUnicode_InternFromString("event_process")) ||
        !(g_unfold_mode = PyUnicode_InternFromString("unfold_mode")) ||
        !(g_classic = PyUnicode_InternFromString("Classic reinterpret")) ||
        !(g_ir_audio = PyUnicode_InternFromString("_ir_audio")) ||
        !(g_img_gray = PyUnicode_InternFromString("_img_gray")) ||
        !(g_max_samps = PyUnicode_InternFromString("space_ir_max_samps")) ||
        !(g_space_ir_on = PyUnicode_InternFromString("space_ir_on")))
        return NULL;
    PyObject* m = PyModule_Create(&kModule);
    if (m) PyModule_AddIntConstant(m, "PRESET_BYTES", (long)sizeof(msg_preset));
    return m;
}
