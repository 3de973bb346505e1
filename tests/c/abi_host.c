/* The C ABI from C (what a cgo shim compiles against):
 * include/cfc.h under a C11 compiler, the pkg/bpf call sequence on a
 * host-only context — create, update with the BPF flags, lookup, walk with
 * get_next_key, bulk dump, delete, close — and the errno conventions. */
#include <errno.h>
#include <stdio.h>
#include <string.h>

#include "cfc.h"

#define CHECK(c)                                                     \
    do {                                                             \
        if (!(c)) {                                                  \
            fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, #c);  \
            return 1;                                                \
        }                                                            \
    } while (0)

/* PolicyKey / PolicyEntry (pkg/maps/policymap/policymap.go:64-80) */
struct policy_key { uint32_t identity; uint16_t dport; uint8_t nexthdr, egress; };
struct policy_entry { uint16_t proxy_port, pad[3]; uint64_t packets, bytes; };

int main(void)
{
    CHECK(cfc_abi_version() == CFC_ABI_VERSION);
    cfc_ctx *ctx = NULL;
    CHECK(cfc_open(CFC_DEVICE_NONE, &ctx) == 0 && ctx);
    int fd = -1, created = 0;
    CHECK(cfc_map_open(ctx, "/sys/fs/bpf/tc/globals/cilium_policy_4112", 1,
                       sizeof(struct policy_key), sizeof(struct policy_entry), 16384, 0,
                       &fd, &created) == 0 && created);
    struct policy_key k = {1000, 0x5000, 6, 0}, k2 = {2, 0, 0, 1}, nk;
    struct policy_entry v = {0}, got;
    CHECK(cfc_map_update(ctx, fd, &k, &v, 0) == 0);
    CHECK(cfc_map_update(ctx, fd, &k, &v, 1 /* BPF_NOEXIST */) == -EEXIST);
    CHECK(cfc_map_update(ctx, fd, &k2, &v, 2 /* BPF_EXIST */) == -ENOENT);
    v.proxy_port = 0x1127;
    CHECK(cfc_map_update(ctx, fd, &k2, &v, 0) == 0);
    CHECK(cfc_map_lookup(ctx, fd, &k2, &got) == 0 && got.proxy_port == 0x1127);
    int n = 0;   /* the DumpWithCallback walk */
    for (int rc = cfc_map_get_next_key(ctx, fd, NULL, &nk); rc == 0;
         rc = cfc_map_get_next_key(ctx, fd, &nk, &nk))
        n++;
    CHECK(n == 2);
    uint64_t cnt = 0;
    CHECK(cfc_map_dump(ctx, fd, NULL, NULL, 0, &cnt) == 0 && cnt == 2);
    struct policy_key keys[2];
    struct policy_entry vals[2];
    CHECK(cfc_map_dump(ctx, fd, keys, vals, 2, &cnt) == 0 && cnt == 2);
    CHECK(cfc_map_delete(ctx, fd, &k) == 0 && cfc_map_delete(ctx, fd, &k) == -ENOENT);
    CHECK(cfc_map_lookup(ctx, fd, &k, &got) == -ENOENT);
    /* no GPU: the datapath half says so */
    CHECK(cfc_commit(ctx, NULL) == -ENODEV);
    CHECK(cfc_strerror(-ENOENT) != NULL);
    CHECK(cfc_map_close(ctx, fd) == 0);
    cfc_close(ctx);
    printf("abi_host: ok\n");
    return 0;
}
