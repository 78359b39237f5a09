/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 * Minimal independent GGUF v2/v3 reader (public container format) for the oracle,
 * so the oracle never shares loader code with the product (csrc/host/gguf.cpp).
 * Reference loader call sites: miocodec.cpp:92-157, :816-853.
 */
#include "gguf_ref.h"

#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

typedef struct {
    const unsigned char *p, *end;
    int ok;
} cur_t;

static int rd(cur_t *c, void *dst, size_t n) {
    if (!c->ok || (size_t)(c->end - c->p) < n) {
        c->ok = 0;
        return 0;
    }
    memcpy(dst, c->p, n);
    c->p += n;
    return 1;
}

static uint64_t rd64(cur_t *c) { uint64_t v = 0; rd(c, &v, 8); return v; }
static uint32_t rd32(cur_t *c) { uint32_t v = 0; rd(c, &v, 4); return v; }

static char *rdstr(cur_t *c) {
    uint64_t n = rd64(c);
    if (!c->ok || (uint64_t)(c->end - c->p) < n) { c->ok = 0; return NULL; }
    char *s = (char *)malloc(n + 1);
    memcpy(s, c->p, n);
    s[n] = 0;
    c->p += n;
    return s;
}

static size_t scalar_size(uint32_t t) {
    switch (t) {
        case 0: case 1: case 7: return 1;
        case 2: case 3: return 2;
        case 4: case 5: case 6: return 4;
        case 10: case 11: case 12: return 8;
        default: return 0;
    }
}

size_t mo_type_size(uint32_t type, int64_t n) {
    switch (type) {
        case 0: return 4 * n;           /* f32 */
        case 1: return 2 * n;           /* f16 */
        case 26: return 4 * n;          /* i32 */
        case 30: return n * 2;          /* bf16 */
        case 2: return n / 32 * 18;     /* q4_0 */
        case 6: return n / 32 * 22;     /* q5_0 */
        case 8: return n / 32 * 34;     /* q8_0 */
        case 12: return n / 256 * 144;  /* q4_K */
        case 14: return n / 256 * 210;  /* q6_K */
        default: return 0;
    }
}

mo_gguf *mo_gguf_open(const char *path) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) return NULL;
    struct stat st;
    if (fstat(fd, &st) != 0) { close(fd); return NULL; }
    void *map = mmap(NULL, st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (map == MAP_FAILED) return NULL;
    mo_gguf *g = (mo_gguf *)calloc(1, sizeof(mo_gguf));
    g->map = map;
    g->size = st.st_size;
    cur_t c = {(const unsigned char *)map, (const unsigned char *)map + st.st_size, 1};
    uint32_t magic = rd32(&c), ver = rd32(&c);
    if (magic != 0x46554747u || (ver != 2 && ver != 3)) { mo_gguf_close(g); return NULL; }
    g->n_tensors = (int)rd64(&c);
    g->n_kv = (int)rd64(&c);
    g->kv = (mo_kv *)calloc(g->n_kv ? g->n_kv : 1, sizeof(mo_kv));
    uint64_t alignment = 32;
    for (int i = 0; i < g->n_kv && c.ok; i++) {
        mo_kv *kv = &g->kv[i];
        kv->key = rdstr(&c);
        kv->type = rd32(&c);
        if (kv->type == 8) {
            kv->str = rdstr(&c);
        } else if (kv->type == 9) {
            uint32_t at = rd32(&c);
            uint64_t n = rd64(&c);
            kv->arr_type = at;
            kv->arr_n = n;
            if (at == 8) {
                kv->arr_str = (char **)calloc(n ? n : 1, sizeof(char *));
                for (uint64_t j = 0; j < n && c.ok; j++) kv->arr_str[j] = rdstr(&c);
            } else {
                size_t es = scalar_size(at);
                if (!es) { c.ok = 0; break; }
                kv->arr_data = c.p;
                if ((uint64_t)(c.end - c.p) < n * es) { c.ok = 0; break; }
                c.p += n * es;
            }
        } else {
            size_t es = scalar_size(kv->type);
            if (!es) { c.ok = 0; break; }
            unsigned char b[8] = {0};
            rd(&c, b, es);
            switch (kv->type) {
                case 0: kv->i = b[0]; break;
                case 1: kv->i = (int8_t)b[0]; break;
                case 2: { uint16_t v; memcpy(&v, b, 2); kv->i = v; } break;
                case 3: { int16_t v; memcpy(&v, b, 2); kv->i = v; } break;
                case 4: { uint32_t v; memcpy(&v, b, 4); kv->i = v; } break;
                case 5: { int32_t v; memcpy(&v, b, 4); kv->i = v; } break;
                case 6: { float v; memcpy(&v, b, 4); kv->f = v; } break;
                case 7: kv->i = b[0] != 0; break;
                case 10: { uint64_t v; memcpy(&v, b, 8); kv->i = (int64_t)v; } break;
                case 11: { int64_t v; memcpy(&v, b, 8); kv->i = v; } break;
                case 12: { double v; memcpy(&v, b, 8); kv->f = v; } break;
            }
        }
        if (kv->key && strcmp(kv->key, "general.alignment") == 0) alignment = (uint64_t)kv->i;
    }
    g->tensors = (mo_tensor *)calloc(g->n_tensors ? g->n_tensors : 1, sizeof(mo_tensor));
    for (int i = 0; i < g->n_tensors && c.ok; i++) {
        mo_tensor *t = &g->tensors[i];
        t->name = rdstr(&c);
        t->n_dims = (int)rd32(&c);
        t->ne[0] = t->ne[1] = t->ne[2] = t->ne[3] = 1;
        for (int d = 0; d < t->n_dims && d < 4; d++) t->ne[d] = (int64_t)rd64(&c);
        t->type = rd32(&c);
        t->offset = rd64(&c);
    }
    if (!c.ok) { mo_gguf_close(g); return NULL; }
    size_t off = (size_t)(c.p - (const unsigned char *)map);
    size_t data0 = (off + alignment - 1) / alignment * alignment;
    for (int i = 0; i < g->n_tensors; i++) {
        mo_tensor *t = &g->tensors[i];
        t->data = (const unsigned char *)map + data0 + t->offset;
        t->nbytes = mo_type_size(t->type, t->ne[0]) * (size_t)(t->ne[1] * t->ne[2] * t->ne[3]);
    }
    return g;
}

void mo_gguf_close(mo_gguf *g) {
    if (!g) return;
    for (int i = 0; i < g->n_kv; i++) {
        free(g->kv[i].key);
        free(g->kv[i].str);
        if (g->kv[i].arr_str) {
            for (uint64_t j = 0; j < g->kv[i].arr_n; j++) free(g->kv[i].arr_str[j]);
            free(g->kv[i].arr_str);
        }
    }
    for (int i = 0; i < g->n_tensors; i++) free(g->tensors[i].name);
    free(g->kv);
    free(g->tensors);
    if (g->map) munmap(g->map, g->size);
    free(g);
}

const mo_kv *mo_gguf_kv(const mo_gguf *g, const char *key) {
    for (int i = 0; i < g->n_kv; i++)
        if (g->kv[i].key && strcmp(g->kv[i].key, key) == 0) return &g->kv[i];
    return NULL;
}

int64_t mo_gguf_int(const mo_gguf *g, const char *key, int64_t def) {
    const mo_kv *kv = mo_gguf_kv(g, key);
    return (kv && kv->type != 6 && kv->type != 12 && kv->type != 8 && kv->type != 9) ? kv->i : def;
}

int64_t mo_gguf_arr_int(const mo_gguf *g, const char *key, int idx, int64_t def) {
    const mo_kv *kv = mo_gguf_kv(g, key);
    if (!kv) return def;
    if (kv->type != 9) return mo_gguf_int(g, key, def);
    if (idx < 0 || (uint64_t)idx >= kv->arr_n || !kv->arr_data) return def;
    const unsigned char *p = (const unsigned char *)kv->arr_data;
    switch (kv->arr_type) {
        case 4: { uint32_t v; memcpy(&v, p + 4 * idx, 4); return v; }
        case 5: { int32_t v; memcpy(&v, p + 4 * idx, 4); return v; }
        case 10: case 11: { int64_t v; memcpy(&v, p + 8 * idx, 8); return v; }
        default: return def;
    }
}

double mo_gguf_float(const mo_gguf *g, const char *key, double def) {
    const mo_kv *kv = mo_gguf_kv(g, key);
    return (kv && (kv->type == 6 || kv->type == 12)) ? kv->f : def;
}

const mo_tensor *mo_gguf_tensor(const mo_gguf *g, const char *name) {
    for (int i = 0; i < g->n_tensors; i++)
        if (strcmp(g->tensors[i].name, name) == 0) return &g->tensors[i];
    return NULL;
}
