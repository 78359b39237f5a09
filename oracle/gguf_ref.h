/* ORACLE — TEST INFRASTRUCTURE ONLY. Minimal GGUF reader for the oracle. */
#ifndef MO_GGUF_REF_H
#define MO_GGUF_REF_H

#include <stddef.h>
#include <stdint.h>

typedef struct {
    char *key;
    uint32_t type, arr_type;
    int64_t i;
    double f;
    char *str;
    uint64_t arr_n;
    char **arr_str;
    const void *arr_data;
} mo_kv;

typedef struct {
    char *name;
    int n_dims;
    int64_t ne[4];
    uint32_t type;
    uint64_t offset;
    size_t nbytes;
    const unsigned char *data;
} mo_tensor;

typedef struct {
    void *map;
    size_t size;
    int n_kv, n_tensors;
    mo_kv *kv;
    mo_tensor *tensors;
} mo_gguf;

mo_gguf *mo_gguf_open(const char *path);
void mo_gguf_close(mo_gguf *g);
const mo_kv *mo_gguf_kv(const mo_gguf *g, const char *key);
int64_t mo_gguf_int(const mo_gguf *g, const char *key, int64_t def);
double mo_gguf_float(const mo_gguf *g, const char *key, double def);
/* element idx of an integer array KV (a scalar KV: its value; absent: def) */
int64_t mo_gguf_arr_int(const mo_gguf *g, const char *key, int idx, int64_t def);
const mo_tensor *mo_gguf_tensor(const mo_gguf *g, const char *name);
size_t mo_type_size(uint32_t type, int64_t n);

#endif
