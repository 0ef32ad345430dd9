/* markstein_check.c (r05, CPU only): is q2 = fma(fma(-q, D, n), rD, q) with q = n * rD and rD = RN(1/D)
 * the correctly rounded n / D? Every numerator significand (2^23) against NDIV divisor significands
 * (the first 64 structured, the rest hashed from SEED); scaling by powers of two is exact, so this covers
 * all quotients whose intermediates stay normal. Build: gcc -O3 -march=native -mfma -ffp-contract=off
 * -fopenmp tools/markstein_check.c -lm; run: ./a.out NDIV SEED. r05: 8192 divisors, 6.9e10 cases, 0 wrong
 * (the uncorrected q: 18.5% wrong). tools/markstein_gpu.hip sweeps all 2^46 pairs on the GPU. */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static float fb(uint32_t u){float f;memcpy(&f,&u,4);return f;}
int main(int argc,char**argv){
  int nd=atoi(argv[1]); unsigned seed=atoi(argv[2]);
  long bad=0, total=0;
  #pragma omp parallel for reduction(+:bad,total) schedule(dynamic)
  for(int k=0;k<nd;k++){
    uint32_t m;
    if(k<64) m = (k==0)?0:(k<24? (1u<<k)-1 : (0x7fffffu>>(k-23)) ^ (k*2654435761u & 0x7fffff));
    else { uint32_t x=(k*2654435761u)^(seed*40503u); x^=x>>13; x*=0x5bd1e995; x^=x>>15; m=x&0x7fffff; }
    float D = fb(0x3f800000u|m);
    volatile float one=1.0f; float rD = one / D;
    for(uint32_t a=0;a<(1u<<23);a++){
      float n = fb(0x3f800000u|a);
      float q = n*rD;
      float r = fmaf(-q, D, n);
      float q2 = fmaf(r, rD, q);
      float ref = n / D;
      bad += (q2 != ref); total++;
    }
  }
  printf("D values %d, tests %ld, mismatches %ld\n", nd, total, bad);
  return 0;
}
