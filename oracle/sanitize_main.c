/*
 * sanitize_main.c -- drives every entry of the CPU restatement once on small
 * seeded inputs, for an AddressSanitizer + UndefinedBehaviorSanitizer build
 * of the oracle ("race detection / sanitizers"):
 *   make -C oracle sanitize && oracle/_san/oracle_san
 * TEST INFRASTRUCTURE ONLY (tests/test_oracle_sanitize.py runs it).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bcn_oracle.h"

static uint32_t rng_state = 0x9E3779B9u;
static uint32_t rnd(void)
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 17;
    rng_state ^= rng_state << 5;
    return rng_state;
}

int main(void)
{
    /* a ragged 2-slice RGBA8 image: gradient + noise, with one transparent corner */
    const uint32_t w = 13, h = 9, s = 2, ch = 4;
    uint8_t *img = (uint8_t *)malloc((size_t)w * h * s * ch);
    for (uint32_t i = 0; i < w * h * s; ++i) {
        const uint32_t x = i % w, y = (i / w) % h;
        for (uint32_t c = 0; c < 3; ++c) img[i * 4 + c] = (uint8_t)((x * 19 + y * 11 + c * 40 + (rnd() & 15)) & 255);
        img[i * 4 + 3] = (x > 8 && y > 5) ? (uint8_t)(rnd() & 255) : 255;
    }
    const uint32_t bx = (w + 3) / 4, by = (h + 3) / 4, nb = bx * by * s;
    uint8_t *out = (uint8_t *)calloc(nb, 16);
    double *err = (double *)calloc(nb, sizeof(double));
    int rc = 0;
    const int fmts[] = {1, 2, 3, 4, 5};
    for (int k = 0; k < 5; ++k) rc |= orc_encode_image(fmts[k], img, w, h, s, ch, 1, -1, -1, 2, out, err);
    rc |= orc_encode_image_bc7(img, w, h, s, ch, 0, 1, 2, 1.0f, 0xFF, out, err);        /* exact search, one row */
    rc |= orc_encode_image_bc7(img, w, h, s, ch, 1, 1, 1, 0.2f, 0xFF, out, err);        /* staged low quality */
    rc |= orc_encode_image_bc7_ex(img, w, h, s, ch, 2, 1, 1, 1.0f, 0xFF, 2, out, err);  /* pruned model */
    rc |= orc_encode_image_bc7_perf(img, w, h, 1, ch, 0, 1, 1, 1.0f, 0xFF, 0.5f, out, err);   /* optQuantTrace_d */
    rc |= orc_encode_image_bc7enc_rows(img, w, h, s, ch, 0, (int32_t)by, 2, 0, 1, out);
    rc |= orc_encode_image_bc7enc(img, w, h, 1, ch, 1, 0, out);
    /* block entries */
    float blk[64];
    uint8_t o16[16];
    for (int i = 0; i < 64; ++i) blk[i] = (float)(rnd() & 255) / 255.0f;
    orc_bc1_block_ex(blk, 2, 0.5f, 1, o16);
    orc_bc4_block(blk, o16);
    orc_rgb4_block(blk, 1, 0, o16);
    orc_explicit_alpha_block(blk, o16);
    (void)orc_bc7_block_ex(blk, 0x30, 1, 0.6f, 1, 1, 1.0f, 0, o16);
    uint8_t rgba[64];
    orc_bc7_decode(o16, rgba);
    /* BC6H: unsigned and signed, HDR values incl. zeros and values past the half range */
    float hdr[4 * 64];
    for (int i = 0; i < 4 * 64; ++i) hdr[i] = (float)(rnd() % 100000) / 997.0f - (i & 64 ? 30.0f : 0.0f);
    for (int i = 0; i < 64; ++i) hdr[i] = 0.0f;
    uint8_t o6[4 * 16];
    float e6[4];
    rc |= orc_encode_bc6h_blocks(hdr, 4, 0, 2, o6, e6);
    rc |= orc_encode_bc6h_blocks(hdr, 4, 1, 1, o6, e6);
    free(img);
    free(out);
    free(err);
    printf("sanitized oracle run: rc=%d\n", rc);
    return rc ? 1 : 0;
}
