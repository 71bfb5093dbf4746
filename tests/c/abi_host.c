/* C-language client of libflcodec.so: the header compiles as C99 and the host-side entry points
 * (no GPU needed) answer like the Python binding does.  Built and run by tests/test_host.py. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "flcodec.h"

int main(void) {
    if (flc_version() != 104) { printf("bad version\n"); return 1; }
    flc_codec_params prm;
    memset(&prm, 0, sizeof(prm));
    prm.codec = FLC_TOPK;
    prm.k = 250000;
    int64_t d = 25000000;
    if (flc_payload_format(&prm) != 5) { printf("topk payload format\n"); return 2; }
    if (flc_payload_bytes(&prm, d) != 16 + 2 * 4 * 250000) { printf("topk payload bytes\n"); return 3; }
    prm.codec = FLC_STD_DITHERING;
    prm.s = 127;
    if (flc_payload_bytes(&prm, d) != 16 + d) { printf("qsgd payload bytes\n"); return 4; }
    if (flc_encode_reduce_workspace_size(&prm, 512, d) == 0) { printf("workspace size\n"); return 5; }
    prm.codec = 99;
    if (flc_encode(&prm, NULL, NULL, 0, NULL, NULL, NULL, NULL, 0, NULL) != FLC_ERR_UNSUPPORTED) {
        printf("unknown codec must be rejected\n");
        return 6;
    }
    if (strlen(flc_last_error_string()) == 0) { printf("no error text\n"); return 7; }
    /* TopK tie rule (flc_codec_params.tie): the zeroed struct selects FLC_TIE_LOWEST; both rules are
     * accepted, anything else is rejected on the host before any device argument is looked at */
    memset(&prm, 0, sizeof(prm));
    prm.codec = FLC_TOPK;
    prm.k = 10;
    if (prm.tie != FLC_TIE_LOWEST || FLC_TIE_HIGHEST != 1) { printf("tie default\n"); return 11; }
    prm.tie = 7;
    if (flc_encode(&prm, NULL, NULL, 0, NULL, NULL, NULL, NULL, 0, NULL) != FLC_ERR_ARG ||
        flc_encode_reduce(&prm, NULL, NULL, 0, NULL, 0, 0, NULL, 1.f, NULL, NULL, NULL, 0, NULL) != FLC_ERR_ARG ||
        strstr(flc_last_error_string(), "tie") == NULL) {
        printf("unknown tie rule must be rejected\n");
        return 12;
    }
    prm.tie = FLC_TIE_HIGHEST;   /* accepted: d = 0 / n = 0 calls succeed without a device */
    if (flc_encode_reduce(&prm, NULL, NULL, 0, NULL, 0, 0, NULL, 1.f, NULL, NULL, NULL, 0, NULL) != FLC_OK) {
        printf("highest-index tie rule rejected\n");
        return 13;
    }
    /* the device-RNG host mirror */
    int64_t idx[10];
    if (flc_device_randk_indices(42, 3, 1000, 10, idx) != 0) { printf("randk indices\n"); return 8; }
    for (int i = 0; i < 10; ++i)
        if (idx[i] < 0 || idx[i] >= 1000) { printf("index range\n"); return 9; }
    double u = flc_device_uniform(42, 3, 7);
    if (!(u >= 0.0 && u < 1.0)) { printf("uniform range\n"); return 10; }
    printf("C ABI host checks OK\n");
    return 0;
}
