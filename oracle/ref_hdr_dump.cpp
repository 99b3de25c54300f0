// TEST INFRASTRUCTURE: harness around the reference HDRLoader (thirdparty/hdrloader),
// linked with the reference's own hdrloader.cpp by oracle/Makefile.  Writes
// int32 width, int32 height, then width*height*3 float32 to argv[2].
#include <stdio.h>
#include "hdrloader.h"
int main(int argc, char** argv) {
  if (argc < 3) return 2;
  HDRLoaderResult res;
  res.width = res.height = 0;
  res.cols = nullptr;
  if (!HDRLoader::load(argv[1], res)) return 1;
  FILE* f = fopen(argv[2], "wb");
  if (!f) return 3;
  fwrite(&res.width, 4, 1, f);
  fwrite(&res.height, 4, 1, f);
  if (res.cols) fwrite(res.cols, 4, (size_t)res.width * res.height * 3, f);
  fclose(f);
  return 0;
}
