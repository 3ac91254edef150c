/*
 * data_types.h -- message element types.
 * Same enumerators and values as the reference include/smi/data_types.h:10-16.
 */
#ifndef SMI_DATA_TYPES_H
#define SMI_DATA_TYPES_H

typedef enum {
    SMI_INT = 1,
    SMI_FLOAT = 2,
    SMI_DOUBLE = 3,
    SMI_CHAR = 4,
    SMI_SHORT = 5
} SMI_Datatype;

#endif /* SMI_DATA_TYPES_H */
