/* test stub (see postgres.h): everything lives in postgres.h */
#include "postgres.h"
