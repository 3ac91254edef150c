/*
 * operation_type.h -- communication operation kinds.
 * Same enumerators and values as include/smi/operation_type.h:11-19 of the
 * reference (there they are carried in the 3-bit op field of the wire header,
 * include/smi/header_message.h:8-27; here they only tag transfers).
 */
#ifndef SMI_OPERATION_TYPE_H
#define SMI_OPERATION_TYPE_H

typedef enum {
    SMI_SEND = 0,
    SMI_RECEIVE = 1,
    SMI_BROADCAST = 2,
    SMI_SYNCH = 3,
    SMI_SCATTER = 4,
    SMI_REDUCE = 5,
    SMI_GATHER = 6
} SMI_Operationtype;

#endif /* SMI_OPERATION_TYPE_H */
