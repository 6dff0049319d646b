/* Host sanitizer run of the C oracle (test infrastructure only): resets and
 * random legal play over several maze configurations, built with
 * -fsanitize=address,undefined by tests/test_oracle_golden.py
 * (test_oracle_under_asan_ubsan).  Any out-of-bounds access, use of freed
 * memory or undefined behaviour in maze_oracle.c aborts the run. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct OEnv OEnv;
OEnv* oenv_new(int n, int size_w, int size_h, int max_t, int difficulty, int rand_start, int rand_sizes, int lo,
               int hi);
void oenv_free(OEnv* e);
void oenv_seed(OEnv* e, int i, uint64_t seed);
int oenv_reset_all(OEnv* e, float* obs, uint8_t* masks);
int oenv_step_all(OEnv* e, const int8_t* act, float* obs, uint8_t* masks, float* reward, uint8_t* done,
                  int auto_reset);

enum { OBS = 65, MASK = 6 };

static uint32_t lcg(uint64_t* s) {
    *s = *s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(*s >> 33);
}

int main(void) {
    /* w, h, max_t, difficulty, rand_start, rand_sizes, lo, hi, steps */
    const int cfgs[][9] = {{10, 10, 1200, 1, 0, 0, 0, 0, 2500}, {20, 20, 1200, 1, 1, 0, 0, 0, 1500},
                           {4, 4, 40, 0, 0, 0, 0, 0, 1500},    {8, 8, 60, 1, 1, 1, 3, 12, 1500},
                           {6, 6, 30, 1, 0, 0, 0, 0, 1500}};
    const int n = 24;
    uint64_t rs = 12345;
    long steps = 0, episodes = 0;
    for (size_t c = 0; c < sizeof(cfgs) / sizeof(cfgs[0]); c++) {
        const int* k = cfgs[c];
        OEnv* e = oenv_new(n, k[0], k[1], k[2], k[3], k[4], k[5], k[6], k[7]);
        for (int i = 0; i < n; i++) oenv_seed(e, i, 1000 * c + i);
        float* obs = malloc(sizeof(float) * n * 2 * OBS);
        uint8_t* masks = malloc((size_t)n * 2 * MASK);
        int8_t* act = malloc((size_t)n * 4);
        float* rew = malloc(sizeof(float) * n);
        uint8_t* done = malloc((size_t)n);
        if (oenv_reset_all(e, obs, masks)) fprintf(stderr, "cfg %zu: generation gave up (Q13)\n", c);
        for (int t = 0; t < k[8]; t++) {
            for (int i = 0; i < n; i++)
                for (int a = 0; a < 2; a++) {
                    const uint8_t* m = masks + (i * 2 + a) * MASK;
                    int legal[5], nl = 0;
                    for (int mv = 0; mv < 5; mv++)
                        if (m[mv]) legal[nl++] = mv;
                    act[(i * 2 + a) * 2] = (int8_t)(nl ? legal[lcg(&rs) % nl] : 4);
                    act[(i * 2 + a) * 2 + 1] = (int8_t)(m[5] && (lcg(&rs) & 1));
                }
            oenv_step_all(e, act, obs, masks, rew, done, 1);
            for (int i = 0; i < n; i++) episodes += done[i];
            steps += n;
        }
        free(obs);
        free(masks);
        free(act);
        free(rew);
        free(done);
        oenv_free(e);
    }
    printf("asan_driver ok: %ld env-steps, %ld episodes\n", steps, episodes);
    return 0;
}
