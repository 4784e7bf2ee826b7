// hostio.h — byte-compatible file formats of gVAMPomi (host C++).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace vio {

// PLINK "FID IID value" rows, std::regex("\\s+") token split
// (src/data.cpp:58-110).  Returns rows read, -1 cannot open, -2 "NA".
int64_t read_phen(const std::string& path, std::vector<double>& y);
// read_phen's standardisation: scale to unit variance, NOT centred
// (src/data.cpp:97-104).  Returns the scale factor.
double standardize_phen(std::vector<double>& y);

// mpi_store_vec_to_file (src/utilities.cpp:241-249): CREATE|WRONLY without
// truncation, M doubles at byte offset S*8.
bool store_vec(const std::string& path, const double* v, int64_t S, int64_t M);
// mpi_read_vec_from_file (src/utilities.cpp:251-267): M doubles from byte S*8;
// missing bytes (short file) read as 0.
bool read_vec(const std::string& path, double* v, int64_t S, int64_t M);

// read_vec_from_file (src/utilities.cpp:104-122): whitespace-separated text,
// values with index [S, S+M); missing ones stay as they are (callers zero).
bool read_text_vec(const std::string& path, double* v, int64_t S, int64_t M);

// setup_io + write_ofile_csv_header (src/vamp.cpp:854-882,
// src/utilities.cpp:388-401): delete, create exclusively, header at offset 0.
bool csv_create_with_header(const std::string& path, const std::vector<std::string>& fields);
// setup_io alone: delete, create exclusively, no header (the probit path
// writes none, src/vamp_probit.cpp)
bool csv_create(const std::string& path);
// write_ofile_csv (src/utilities.cpp:366-385): "%5d" + n x ", %20.15f" + "\n"
// at byte offset it * strlen(row).
bool csv_write_row(const std::string& path, int it, const double* vals, int n);
std::string csv_format_row(int it, const double* vals, int n);

// Rendezvous file of a multi-process CLI job (replaces mpirun's bootstrap):
// rank 0 publishes the RCCL id, the other ranks fetch it.  The file carries a
// run nonce (VAMPOMI_RUN_ID, torchrun's TORCHELASTIC_RUN_ID, the MPI / PMIx
// job namespace, slurm's job.step, else MASTER_ADDR:MASTER_PORT); a reader
// accepts only a file with its own nonce.  Without any of them: only a file
// written after not_before (seconds since the epoch) whose id is still there,
// unchanged, 3 s later (rank 0 of a new job replaces a stale file as it
// starts).  Rank 0 removes the file once the communicator is up (rdzv_remove).
std::string rdzv_nonce();
bool rdzv_publish(const std::string& path, const std::string& nonce, const void* id, int nbytes);
bool rdzv_fetch(const std::string& path, const std::string& nonce, double not_before, void* id, int nbytes,
                int timeout_ms);
void rdzv_remove(const std::string& path);

}  // namespace vio
