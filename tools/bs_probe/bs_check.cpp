#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include "bitslice_aes.h"
extern "C" {
#include "aesgcm_oracle.h"
}
using namespace ptls_hip;
static uint8_t gmul(uint8_t a, uint8_t b){uint8_t p=0;while(b){if(b&1)p^=a;a=(a<<1)^((a&0x80)?0x1b:0);b>>=1;}return p;}
int main(){
  uint8_t S[256];
  for(int x=0;x<256;x++){uint8_t inv=0; for(int y=1;y<256;y++) if(gmul(x,y)==1) inv=y; uint8_t s=inv, r=inv; for(int i=0;i<4;i++){r=(r<<1)|(r>>7); s^=r;} S[x]=s^0x63;}
  int bad=0;
  for(int g=0; g<8; g++){ uint32_t P[8]={0}; for(int k=0;k<32;k++){int x=g*32+k; for(int j=0;j<8;j++) if((x>>j)&1) P[j]|=1u<<k;}
    bs::sbox<0>(P); for(int k=0;k<32;k++){int x=g*32+k; int y=0; for(int j=0;j<8;j++) y|=((P[j]>>k)&1)<<j; if(y!=S[x]){bad++; if(bad<5) printf("sbox %02x -> %02x want %02x\n",x,y,S[x]);}}}
  printf("sbox mismatches: %d\n", bad);
  srand(1);
  for(int kl=16; kl<=32; kl+=16){
    uint8_t key[32], rkb[240]; for(int i=0;i<32;i++) key[i]=rand();
    int rounds = oracle_aes_expand(key, kl, rkb);
    uint32_t rk[60]; memcpy(rk, rkb, 240);
    uint8_t blk[32][16]; for(int k=0;k<32;k++) for(int i=0;i<16;i++) blk[k][i]=rand();
    uint32_t P[128]; for(int k=0;k<32;k++) for(int w=0;w<4;w++) memcpy(&P[32*w+k], &blk[k][4*w], 4);
    bs::transpose_all(P);
    if (rounds==10) bs::encrypt<10>(P, rk); else bs::encrypt<14>(P, rk);
    bs::transpose_all(P);
    int m=0; for(int k=0;k<32;k++){ uint8_t exp[16], got[16]; oracle_aes_encrypt(rkb, rounds, blk[k], exp); for(int w=0;w<4;w++) memcpy(&got[4*w], &P[32*w+k], 4); if(memcmp(exp,got,16)) m++; }
    printf("aes-%d (rounds %d): %d/32 mismatches\n", kl*8, rounds, m);
  }
}
