/* ddt_oracle.c placeholder filled below */
